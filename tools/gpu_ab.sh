# A/B of env-var knobs: grid parity tests once, then per setting the stamps breakdown and the headline bench.
#   bash tools/gpu_ab.sh "A=1,B=2 A=0 ..."   (SKIP_TESTS=1 to skip the tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -m pytest tests/test_grid_gpu.py tests/test_shard_gpu.py -q -x > gpurun_out/t.log 2>&1; rc=$?
  grep -E "FAILED|passed|failed|Error" gpurun_out/t.log | head -20; [ $rc -eq 0 ] || exit $rc
fi
for v in $1; do
  echo "== $v"
  E=$(echo $v | tr , " ")
  env $E timeout -k 10 120 python tools/stamps.py 1048576 > gpurun_out/stamps_$v.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/stamps_$v.log; exit 1; }
  grep -v amdgpu gpurun_out/stamps_$v.log | head -11
  env $E timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/bench_$v.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'])"
done
