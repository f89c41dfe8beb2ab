"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for kernels matching a name."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, pat = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for fn in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(fn) as f:
        for row in csv.DictReader(f):
            if pat in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} n={len(v):4d} mean={sum(v)/len(v):.6g}")
