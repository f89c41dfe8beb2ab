# C-ROOMS: GPU parity/law tests (ziggurat normals) and the configs[4] bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cr
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crooms_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 400 python bench.py --workload crooms --steps 512 --warmup 64 --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print('crooms value %.4e'%d['value'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'], 'frac %.3f'%d['roofline']['frac'])"
