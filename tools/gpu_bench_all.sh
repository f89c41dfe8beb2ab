# GPU tests of the non-grid backends + bench lines of the four single-GPU workloads (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -m pytest tests/test_anttag_gpu.py tests/test_crooms_gpu.py tests/test_taxi_gpu.py -q -x > gpurun_out/t2.log 2>&1; rc=$?
  grep -E "FAILED|passed|failed|Error" gpurun_out/t2.log | head -20; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WORKLOADS:-anttag crooms taxi fourrooms}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-256} --warmup 64 --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/bench_$w.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$w.log').read().strip().splitlines()[-1]); print('$w', 'value %.4e'%d['value'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'])"
done
