# Round 2, call B: launch-prologue rework (one LDS image copy, role loads overlapping it, atomic metrics):
# grid + bench-path parity tests, latency probe, stamps at K = 20 / 128, driver-config bench, VALU microbench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2b
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 $PT tests/test_bench_path_gpu.py tests/test_grid_gpu.py tests/test_device_error_gpu.py tests/test_shard_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/tests.log
timeout -k 10 60 ./tools/mb_valu.bin > $O/mb_valu.log 2>&1 || { echo MB_FAIL; tail -5 $O/mb_valu.log; exit 1; }
cat $O/mb_valu.log
timeout -k 10 180 python -u tools/latency_probe.py 1048576 1 20 128 > $O/lat.log 2>&1 || { echo LAT_FAIL; tail -20 $O/lat.log; exit 1; }
grep -v amdgpu.ids $O/lat.log
timeout -k 10 120 python tools/stamps.py 1048576 20 > $O/stamps20.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/stamps20.log; exit 1; }
grep -v amdgpu.ids $O/stamps20.log | head -4
timeout -k 10 120 python tools/stamps.py 1048576 128 > $O/stamps128.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/stamps128.log; exit 1; }
grep -v amdgpu.ids $O/stamps128.log | head -12
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_driver.log; exit 1; }
tail -n 1 $O/bench_driver.log | cut -c 1-600
echo R2B_OK
