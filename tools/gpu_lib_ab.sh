# In-call A/B of two library builds (current vs libgympo_amd_ab.so from tools/build_rev_lib.sh) on one box.
#   WORKLOADS="crooms ..." bash tools/gpu_lib_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for W in ${WORKLOADS:-fourrooms}; do
    for L in libgympo_amd.so libgympo_amd_ab.so; do
      GYM_PO_AMD_LIB=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd/$L timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-256} --warmup 64 --no-cpu-baseline > gpurun_out/ab_${W}_$L.log 2>&1 || { echo "bench $W $L failed"; tail -5 gpurun_out/ab_${W}_$L.log; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab_${W}_$L.log').read().strip().splitlines()[-1]); print('$rep $W $L', 'value %.4e'%d['value'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'])"
    done
  done
done
