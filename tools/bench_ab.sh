# In-call A/B of bench.py lines across library variants (tools/build_variant.sh):
#   bash tools/bench_ab.sh "base w3" [bench args, e.g. --workload crooms]
set -eo pipefail
mkdir -p gpurun_out/bab
LD=$PWD/gym-po-taxi_amd/gym_po_amd
VARS=$1
shift
for rep in 1 2; do
  for V in $VARS; do
    L=$LD/libgympo_amd_$V.so
    [ "$V" = base ] && L=$LD/libgympo_amd.so
    GYM_PO_AMD_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bab/$V.log 2>&1
    echo "== $rep $V $(tail -n 1 gpurun_out/bab/$V.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["frac"], r["kernel_avg_us"])')"
  done
done
