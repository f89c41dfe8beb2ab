"""Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on this GPU with a plain device copy of known size (the
bench's PMC correction doubles FETCH_SIZE for wide coalesced reads, MI355X_MICROARCH.md HBM/rocprofv3 section).
Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`; the copy kernel reads and writes N bytes."""
import torch

N = 1 << 28  # 256 MiB, well past the 256 MB Infinity Cache when the two buffers are counted
a = torch.ones(N, dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
print("copied", N, "bytes x3")
