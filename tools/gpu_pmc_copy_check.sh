# FETCH_SIZE / WRITE_SIZE of a 256 MiB device copy (tools/pmc_copy_check.py), one counter per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmccopy
mkdir -p $O
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $O/$P -o p -- python3 tools/pmc_copy_check.py > $O/$P.log 2>&1 || { echo FAIL $P; tail -20 $O/$P.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for P in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"gpurun_out/pmccopy/{P}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    names = {}
    for r in rows:
        if r.get("Counter_Name") == P:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
    for d in sorted(per, key=int):
        print(P, d, names[d], "%.0f KiB" % per[d], "= %.3f x 256 MiB" % (per[d] * 1024 / (1 << 28)))
PY
