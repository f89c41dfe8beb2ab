# Grid / bench-path / device-error / shard GPU tests of the current build (fast parity gate after a kernel change).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_path_gpu.py tests/test_grid_gpu.py tests/test_device_error_gpu.py tests/test_shard_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
