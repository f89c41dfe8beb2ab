# Round 2, call C: bench-path parity tests on the new build, then an in-call A/B (HEAD lib vs new) of
# the latency probe (K = 1, 20, 128) and the driver-config bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2c
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_bench_path_gpu.py tests/test_grid_gpu.py tests/test_device_error_gpu.py tests/test_shard_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
for rep in 1 2; do
  for L in libgympo_amd_ab.so libgympo_amd.so; do
    GYM_PO_AMD_LIB=$LD/$L timeout -k 10 120 python -u tools/latency_probe.py 1048576 1 20 128 > $O/lat_$L.log 2>&1 || { echo LAT_FAIL; tail -20 $O/lat_$L.log; exit 1; }
    echo "== $rep $L"; grep "B=" $O/lat_$L.log
    GYM_PO_AMD_LIB=$LD/$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$L.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/b_$L.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); print('bench --steps 20: value %.4e'%d['value'], 'kernel_us %.1f'%d['roofline']['kernel_avg_us'])"
  done
done
