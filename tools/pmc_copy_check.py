"""Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on this GPU with a plain device copy of known size (the
bench's PMC correction doubles FETCH_SIZE for wide coalesced reads, MI355X_MICROARCH.md HBM/rocprofv3 section).
Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`; the copy kernel reads and writes N bytes."""
import collections
import csv
import glob
import sys

N = 1 << 28  # 256 MiB, well past the 256 MB Infinity Cache when the two buffers are counted


def summarize(root):
    """Per-dispatch counter totals of the two passes (tools/gpu.sh copycal) as multiples of the copied bytes."""
    for P in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = []
        for f in glob.glob(f"{root}/{P}/**/*counter_collection.csv", recursive=True):
            rows += list(csv.DictReader(open(f)))
        per, names = collections.defaultdict(float), {}
        for r in rows:
            if r.get("Counter_Name") == P:
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
        for d in sorted(per, key=int):
            print(P, d, names[d], "%.0f KiB" % per[d], "= %.3f x 256 MiB" % (per[d] * 1024 / N))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        import torch
        a = torch.ones(N, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        print("copied", N, "bytes x3")
