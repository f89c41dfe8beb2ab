"""Attribute the host-side time of bench.py's timed call (VERDICT r2 "next" #3) from a rocprofv3
`--kernel-trace --hip-runtime-trace` capture of `bench.py --steps 20 --warmup 5` (tools/gpu.sh hiptrace):
for each fused-kernel launch, host hipLaunchKernel entry -> return, GPU kernel begin -> end, and the
synchronize that waited for it.

    python tools/host_gap.py gpurun_out/hiptrace/out [kernel_substring]
"""
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "grid_rollout_numpy"
api = list(csv.DictReader(open(glob.glob(os.path.join(root, "*hip_api_trace.csv"))[0])))
ker = list(csv.DictReader(open(glob.glob(os.path.join(root, "*kernel_trace.csv"))[0])))
by_corr = {r["Correlation_Id"]: r for r in api}
syncs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api
               if r["Function"] in ("hipDeviceSynchronize", "hipStreamSynchronize", "hipEventSynchronize"))
rows = []
for k in sorted(ker, key=lambda r: int(r["Start_Timestamp"])):
    if pat not in k["Kernel_Name"]:
        continue
    a = by_corr.get(k["Correlation_Id"])
    if a is None:
        continue
    l0, l1 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    k0, k1 = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    s = next(((s0, s1, f) for s0, s1, f in syncs if s1 >= k1 and s0 <= k1 + 1_000_000), None)
    prev_sync_end = max((s1 for s0, s1, f in syncs if s1 <= l0), default=None)
    rows.append((l0, l1, k0, k1, s, prev_sync_end))
print(f"{len(rows)} launches of {pat} (times in us)")
print(" #  prev sync end -> launch call | launch call | call return -> kernel begin | kernel | kernel end -> "
      "sync return | sync fn")
for i, (l0, l1, k0, k1, s, ps) in enumerate(rows):
    pre = (l0 - ps) / 1e3 if ps else float("nan")
    post = (s[1] - k1) / 1e3 if s else float("nan")
    print(f"{i:2d} {pre:10.2f} {(l1 - l0) / 1e3:10.2f} {(k0 - l1) / 1e3:10.2f} {(k1 - k0) / 1e3:10.2f} {post:10.2f}  "
          f"{s[2] if s else '-'}")
