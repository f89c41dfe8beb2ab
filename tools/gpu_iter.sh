# One build->measure iteration on the GPU box: grid parity tests, phase stamps, headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_grid_gpu.py -q -x > gpurun_out/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamps.py 1048576 > gpurun_out/stamps.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/stamps.log; exit 1; }
tail -8 gpurun_out/stamps.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print('value %.3e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.2f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'], 'spl', d['roofline']['steps_per_launch'])"
