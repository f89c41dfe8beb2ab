# Round 2, call D: final prologue build (one LDS image copy at the top, by-value params, atomic metrics):
# bench-path parity tests, A/B vs HEAD lib (latency probe), driver-config bench with/without device
# kernargs, stamps at K = 20.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2d
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_bench_path_gpu.py tests/test_grid_gpu.py tests/test_device_error_gpu.py tests/test_shard_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
for rep in 1 2; do
  for L in libgympo_amd_ab.so libgympo_amd.so; do
    for KA in 0 1; do
      HIP_FORCE_DEV_KERNARG=$KA GYM_PO_AMD_LIB=$LD/$L timeout -k 10 120 python -u tools/latency_probe.py 1048576 1 20 128 > $O/lat.log 2>&1 || { echo LAT_FAIL; tail -20 $O/lat.log; exit 1; }
      echo "== $rep $L KERNARG=$KA"; grep "B=" $O/lat.log | sed 's/host wall median/wall/; s/(p10 [0-9.]*); //'
    done
  done
  for KA in 0 1; do
    HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/b.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('bench --steps 20 KERNARG=$KA: value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'])"
  done
done
timeout -k 10 120 python tools/stamps.py 1048576 20 > $O/stamps20.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/stamps20.log; exit 1; }
grep -v amdgpu.ids $O/stamps20.log | head -4
