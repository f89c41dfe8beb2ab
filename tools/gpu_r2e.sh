# Round 2, call E: deferred resetter cells + VALU trims: grid / bench-path parity tests on the default
# build, then in-call A/B of the variants (latency probe, kernel-event time per launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2e
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_bench_path_gpu.py tests/test_grid_gpu.py tests/test_device_error_gpu.py tests/test_shard_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
VARS="ab v00 v10 v01 v11" KS="1 20 128" bash tools/gpu_var_ab.sh
