"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for each kernel matching a name."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, pats = sys.argv[1], sys.argv[2:]
vals = defaultdict(lambda: defaultdict(list))
for fn in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(fn) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            for pat in pats:
                if pat in name:
                    vals[pat][row["Counter_Name"]].append(float(row["Counter_Value"]))
for pat in pats:
    print(f"== {pat}")
    d = {k: sum(v) / len(v) for k, v in vals[pat].items()}
    for k in sorted(d):
        print(f"   {k:28s} n={len(vals[pat][k]):4d} mean={d[k]:.6g}")
    w = d.get("SQ_WAVES")
    if w:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                  "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
            if k in d:
                print(f"   per-wave {k:24s} {d[k] / w:10.1f}")
