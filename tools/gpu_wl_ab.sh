# In-call A/B of library variants on one bench workload: WL=crooms VARS="ab zc zo" bash tools/gpu_wl_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wl
mkdir -p $O
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
for rep in 1 2; do
  for V in $VARS; do
    GYM_PO_AMD_LIB=$LD/libgympo_amd_$V.so timeout -k 10 300 python bench.py --workload $WL --steps ${STEPS:-256} --warmup 64 --no-cpu-baseline > $O/b_$V.log 2>&1 || { echo BENCH_FAIL $V; tail -20 $O/b_$V.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$V.log').read().strip().splitlines()[-1]); print('$rep $WL $V value %.4e'%d['value'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
