# Round 2, call A: the new parity tests (bench path, device error, taxi one-hot), the full -m gpu suite,
# the driver-config bench line, a steady-state line, and launch-level stamps at K = 20 / 128.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2a
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_bench_path_gpu.py tests/test_device_error_gpu.py tests/test_taxi_gpu.py > $O/new_tests.log 2>&1 || { echo NEWTESTS_FAIL; tail -60 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
timeout -k 10 900 $PT tests -m gpu > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_2000.log 2>&1 || { echo BENCH2_FAIL; tail -30 $O/bench_2000.log; exit 1; }
tail -1 $O/bench_2000.log
timeout -k 10 120 python tools/stamps.py 1048576 20 > $O/stamps20.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/stamps20.log; exit 1; }
head -5 $O/stamps20.log
timeout -k 10 120 python tools/stamps.py 1048576 128 > $O/stamps128.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/stamps128.log; exit 1; }
cat $O/stamps128.log
echo R2A_OK
