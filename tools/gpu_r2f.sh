# Round 2, call F: full -m gpu suite + smoke on the current build; small-B (strong-scaling shard sizes)
# fused-kernel lines at 2^17 / 2^18 envs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
for B in 131072 262144; do
  timeout -k 10 300 python bench.py --envs $B --steps 1024 --warmup 128 --no-cpu-baseline > $O/b_$B.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/b_$B.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$B.log').read().strip().splitlines()[-1]); print('B=$B value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'steps/launch', d['roofline']['steps_per_launch'], 'frac %.3f'%d['roofline']['frac'])"
done
