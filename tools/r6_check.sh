# Round-6 GPU check: windowed-kernel parity tests, an in-call A/B of the round-5 library (libgympo_amd_r5.so,
# tools/build_commit_variant.sh r5 <commit>) against the current one, the driver's bench command, and the
# launch-footprint probe. Every GPU step under its own limit; the first failure ends the call.
#   bash tools/r6_check.sh [tests|ab|bench|floor]...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6
mkdir -p $O
LD=$PWD/gym-po-taxi_amd/gym_po_amd
run() {
  local t=$1 log=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1 || { echo "FAIL ($?): $*"; tail -40 "$log"; exit 1; }
}
for task in "${@:-tests ab bench floor}"; do
  case $task in
    tests)
      run 600 $O/tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread ${TESTS:-tests/test_wgrid_gpu.py tests/test_bench_path_gpu.py} -m gpu
      tail -n 1 $O/tests.log ;;
    ab)
      for rep in 1 2; do
        for V in r5 base; do
          L=$LD/libgympo_amd_$V.so
          [ "$V" = base ] && L=$LD/libgympo_amd.so
          GYM_PO_AMD_LIB=$L GP_KNOBS=wg_kmax=1000 run 150 $O/lat_$V.log python -u tools/latency_probe.py 1048576 ${ABK:-20 128}
          echo "== $rep $V"; grep "B=" $O/lat_$V.log
        done
      done ;;
    tmodes)  # in-call A/B of timing-study schedules of the current library (wg_tmode bits, csrc/wgrid.hip TM_*)
      for rep in 1 2; do
        for T in ${TMODES:-0 4096 64 4160 8 256}; do
          GP_KNOBS=wg_kmax=1000,wg_tmode=$T run 150 $O/tm_$T.log python -u tools/latency_probe.py 1048576 ${ABK:-20 128}
          echo "== $rep tmode $T"; grep "B=" $O/tm_$T.log
        done
      done ;;
    bench)
      for rep in 1 2; do
        run 300 $O/bench_$rep.log python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
        tail -n 1 $O/bench_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("bench", d["value"], d["ms_per_step"], r["frac"], r["kernel_avg_us"], r["kernel"], d["config"]["kernel_autotune"])'
      done ;;
    stamps)  # phase stamps of the windowed kernel (the GP_STAMPS library, built beforehand on the CPU)
      for K in ${STK:-64 20}; do
        GYM_PO_AMD_LIB=$LD/libgympo_amd_stamps.so run 200 $O/wstamps_k$K.log python -u tools/wstamps.py 1048576 $K
        cat $O/wstamps_k$K.log
      done ;;
    floorprof)  # the launch-footprint probe under rocprofv3 (dispatch-timestamp durations of the same launches)
      run 300 $O/floorprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/floorprof -o p -- python3 -u tools/launch_floor.py 60
      for f in $(find $O/floorprof -name "*kernel_stats.csv"); do cp $f $O/floor_kernel_stats.csv; cat $f; done ;;
    taxiprof)  # per-kernel time of seed-identical Taxi at 65,536 and 4M envs (rocprofv3 kernel trace)
      run 400 $O/taxiprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/taxiprof -o p -- python3 -u tools/taxi_numpy_rate.py ${TAXI_B:-65536 4194304}
      grep numpy $O/taxiprof.log
      for f in $(find $O/taxiprof -name "*kernel_stats.csv"); do cp $f $O/taxi_kernel_stats.csv; head -12 $f | cut -c1-220; done ;;
    fsimd)  # windowed kernel: per-SIMD window-row deltas (wg_fill_simd, 4 signed nibbles), LIB:CODE cases
      for rep in 1 2; do
        for c in ${FS_CASES:-base:0}; do
          IFS=: read V F <<< "$c"
          L=$LD/libgympo_amd_$V.so
          [ "$V" = base ] && L=$LD/libgympo_amd.so
          GYM_PO_AMD_LIB=$L GP_KNOBS=wg_kmax=1000,wg_fill_simd=$F run 150 $O/fs_${V}_$F.log python -u tools/latency_probe.py ${FS_B:-1048576} ${ABK:-20 128}
          echo "== $rep $V fill_simd $F"; grep "B=" $O/fs_${V}_$F.log
        done
      done ;;
    strong)  # strong-scaling shard sizes: the fused kernel (wg_kmax 0) vs the windowed kernel (wg_kmax 1000)
      for B in ${STRONG_B:-131072 262144}; do
        for kn in 0 1000; do
          GP_KNOBS=wg_kmax=$kn run 150 $O/strong_${B}_$kn.log python -u tools/latency_probe.py $B 20 128
          echo "== B $B wg_kmax $kn"; grep "B=" $O/strong_${B}_$kn.log
        done
      done ;;
    blocks)  # windowed kernel block size at a shard size (wg_block_envs knob): envs per block E -> G = B / E blocks
      for E in ${BLK_E:-512 1024 2048}; do
        GP_KNOBS=wg_kmax=1000,wg_block_envs=$E run 150 $O/blk_$E.log python -u tools/latency_probe.py ${BLK_B:-131072} 20 128
        echo "== E $E"; grep "B=" $O/blk_$E.log
      done ;;
    persist)  # the streaming rollouts' persistent grid: balanced_grid's choice (bpc 0) vs forced blocks per CU
      for W in ${PW:-crooms anttag taxi}; do
        for rep in 1 2; do
          for bpc in ${PBPC:-0 5 4}; do
            GP_KNOBS=persist_bpc=$bpc run 300 $O/persist_${W}_$bpc.log python3 bench.py --no-cpu-baseline --workload $W ${PSTEPS:---steps 1024 --warmup 128}
            tail -n 1 $O/persist_${W}_$bpc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("'$W' bpc '$bpc'", "%.4g" % d["value"], "us/step %.3f" % (d["ms_per_step"]*1e3), "frac %.3f" % r["frac"], d["config"].get("persistent_grid"))'
          done
        done
      done ;;
    occ)  # streaming rollouts: library variant (occupancy build) x forced blocks per CU, "W:LIB:BPC" cases
      for rep in 1 2; do
        for c in ${OCC_CASES:-crooms:base:0 crooms:base:8 crooms:cw6:0 crooms:cw8:0 anttag:base:0 anttag:base:8 anttag:at8:0}; do
          IFS=: read W V bpc <<< "$c"
          L=$LD/libgympo_amd_$V.so
          [ "$V" = base ] && L=$LD/libgympo_amd.so
          GYM_PO_AMD_LIB=$L GP_KNOBS=persist_bpc=$bpc run 300 $O/occ_${W}_${V}_$bpc.log python3 bench.py --no-cpu-baseline --workload $W --steps 1024 --warmup 128
          tail -n 1 $O/occ_${W}_${V}_$bpc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("'$c'", "%.4g" % d["value"], "us/step %.3f" % (d["ms_per_step"]*1e3), "frac %.3f" % r["frac"], d["config"].get("persistent_grid"))'
        done
      done ;;
    xg)  # C-ROOMS exact mode per knob set (XG_CASES: ';'-separated GP_KNOBS values, '-' = none) at XG_B envs
      for rep in 1 2; do
        IFS=';' read -ra CS <<< "${XG_CASES:--;xg_ppt_min=64;xg_ppt_min=64,xg_spb_min=64}"
        for c in "${CS[@]}"; do
          kn=$c; [ "$c" = "-" ] && kn=""
          GP_KNOBS=$kn MODES=numpy run 300 $O/xg.log python3 -u tools/crooms_numpy_rate.py ${XG_B:-65536}
          echo "== $rep [$c]"; cat $O/xg.log | grep numpy
        done
      done ;;
    valu)  # VALU issue rates (tools/mb_valu.hip, built beforehand)
      run 120 $O/valu.log tools/mb_valu.bin
      cat $O/valu.log ;;
    counters)  # the PMC counters this GPU offers
      run 120 $O/counters.log rocprofv3 -L
      grep -i -E "icache|ifetch|SQC_" $O/counters.log | head -60 ;;
    floor)
      run 200 $O/floor.log python -u tools/launch_floor.py 200
      cat $O/floor.log ;;
  esac
done
