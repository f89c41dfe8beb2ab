set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_grid_gpu.py tests/test_shard_gpu.py -q -x > gpurun_out/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/t.log | head; [ $rc -eq 0 ] || exit $rc
for c in 64 128 256 64; do
  timeout -k 10 300 python bench.py --steps 2048 --warmup 256 --chunk $c --no-cpu-baseline > gpurun_out/bench_c$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_c$c.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_c$c.log').read().strip().splitlines()[-1]); print('chunk $c', 'value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'])"
done
