"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<config>.json for bench.py.

    python tools/pmc_to_json.py <pmc_root> <kernel_substring> <config_key> <out.json> <workload> <steps_per_launch>

Every profiled dispatch must have the same launch shape (run bench.py with --chunk C and --steps/--warmup
multiples of C): the record is keyed on steps_per_launch, and bench.py only reuses it for lines of that
shape (or fits T(K) = fixed + per_step*K over records at several shapes).

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so it is doubled.
Both come from separate --pmc passes (TCC slots cannot hold both at once).
"""
import csv
import glob
import hashlib
import json
import os
import sys

root, pat, cfg, out, workload = sys.argv[1:6]
steps_per_launch = float(sys.argv[6])
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
for fn in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(fn) as f:
        rows = [r for r in csv.DictReader(f) if pat in r.get("Kernel_Name", "") and r["Counter_Name"] in vals]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))  # launch order (the same in every pass)
    for r in rows:
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
if not vals["FETCH_SIZE"] or not vals["WRITE_SIZE"]:
    sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for {pat!r} under {root}")
# A bench command launches a few shorter warmup chunks (1 and W - 1 steps) before its C-step launches: keep the
# launches whose WRITE_SIZE is within 5% of the median (the C-step ones), and the same launches of the FETCH pass
# (the passes run the same command, so launch i is the same launch in both).
import statistics  # noqa: E402
med = statistics.median(vals["WRITE_SIZE"])
keep = [i for i, v in enumerate(vals["WRITE_SIZE"]) if abs(v - med) <= 0.05 * med]
if len(vals["FETCH_SIZE"]) == len(vals["WRITE_SIZE"]):
    vals = {k: [v[i] for i in keep] for k, v in vals.items()}
else:  # the passes launched different sequences (e.g. an autotuned kernel choice): filter each on its own median
    for k in vals:
        m = statistics.median(vals[k])
        vals[k] = [v for v in vals[k] if abs(v - m) <= 0.05 * m]
fetch_kib = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write_kib = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(here, "gym-po-taxi_amd", "gym_po_amd", "libgympo_amd.so"), "rb") as f:
    h = hashlib.sha1(f.read()).hexdigest()[:12]
sys.path.insert(0, here)
import bench  # noqa: E402
d = {"config": cfg, "kernel": pat, "lib_hash": h, "src_hash": bench.src_hash(workload),
     "steps_per_launch": steps_per_launch,
     "dispatches": {"FETCH_SIZE": len(vals["FETCH_SIZE"]), "WRITE_SIZE": len(vals["WRITE_SIZE"])},
     "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
     "hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
     "correction": "FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads), KiB -> bytes"}
with open(out, "w") as f:
    json.dump(d, f, indent=1)
print(json.dumps(d))
