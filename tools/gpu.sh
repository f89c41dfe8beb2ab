# One parameterised GPU-box helper (run through gpurun from the repo root). Every GPU step has its own
# time limit; the first failure ends the call (set -e + explicit exits). Output lands in gpurun_out/<task>/.
#
#   bash tools/gpu.sh tests [pytest args]      -m gpu suite (or the given test files) + smoke
#   bash tools/gpu.sh bench [bench args]       one bench.py line (no CPU baseline unless CPU=1)
#   bash tools/gpu.sh prof [bench args]        rocprofv3 --kernel-trace --stats of a bench command
#   bash tools/gpu.sh hiptrace [bench args]    the same with --hip-runtime-trace (host-side attribution)
#   bash tools/gpu.sh pmc [bench args]         FETCH_SIZE and WRITE_SIZE passes -> gpurun_out/pmc/pmc.json
#   bash tools/gpu.sh sq [bench args]          SQ counter passes (VALU / LDS / waits per wave)
#   bash tools/gpu.sh stamps [B K]             phase stamps of the fused numpy kernel (GP_STAMPS build)
#   bash tools/gpu.sh ab "V1 V2 ..." [B K...]  in-call A/B of library variants (tools/build_variant.sh) at K steps
#   bash tools/gpu.sh copycal                  FETCH_SIZE / WRITE_SIZE calibration on a plain device copy
#   bash tools/gpu.sh measure                 driver-config + steady headline lines, MEASURE_WL workloads, VALU costs,
#                                              CRATE="B ..." C-ROOMS exact-mode rates
#   bash tools/gpu.sh multi                    bench.py's N>1 path with 2 gloo ranks on one GPU
# Env: PMC_KERNEL / PMC_CFG / PMC_WORKLOAD for pmc (defaults: the headline kernel and config); PMCSET_ONLY="crooms .."
#      limits pmcset to those workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
task=$1
shift || true
O=gpurun_out/$task
mkdir -p $O
run() {  # run <seconds> <log> <cmd...>: one GPU step under its own limit; stop the call on failure
  local t=$1 log=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1 || { echo "FAIL ($?): $*"; tail -30 "$log"; exit 1; }
}
last_json() { python3 -c "import json,sys; print(json.dumps(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]))[:${2:-1500}])" "$1"; }
case "$task" in
  tests)
    run 1000 $O/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread ${@:-tests} -m gpu
    tail -n 1 $O/tests.log
    run 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
    tail -n 1 $O/smoke.log ;;
  bench)
    run 600 $O/bench.log python3 bench.py $([ -z "$CPU" ] && echo --no-cpu-baseline) "$@"
    last_json $O/bench.log 2500 ;;
  prof)
    run 300 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/out -o p -- python3 bench.py --no-cpu-baseline "$@"
    for f in $(find $O/out -name "*kernel_stats.csv"); do cp $f $O/kernel_stats.csv; head -8 $f; done
    last_json $O/prof.log 800 ;;
  hiptrace)
    run 300 $O/trace.log rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/out -o p -- python3 bench.py --no-cpu-baseline "$@"
    for f in $(find $O/out -name "*stats.csv"); do cp $f $O/$(basename $f); done
    ls $O ;;
  pmc)
    i=0
    for C in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      run 300 $O/p$i.log rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p -- python3 bench.py --no-cpu-baseline "$@"
    done
    python3 tools/pmc_to_json.py $O ${PMC_KERNEL:-grid_rollout_numpy} ${PMC_CFG:-fourrooms_hansen4_B1048576_numpy} $O/pmc.json ${PMC_WORKLOAD:-fourrooms} ${PMC_K:-20}
    cat $O/pmc.json ;;
  sq)
    i=0
    for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA"; do
      i=$((i+1))
      run 240 $O/p$i.log rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p -- python3 bench.py --no-cpu-baseline "$@"
    done
    python3 tools/pmc_summary.py $O ${SQ_KERNELS:-grid_rollout_numpy grid_rollout_counter crooms_rollout anttag_rollout taxi_rollout} ;;
  stamps)
    run 120 $O/stamps.log python tools/stamps.py ${1:-1048576} ${2:-128}
    grep -v amdgpu.ids $O/stamps.log ;;
  knobab)  # in-call A/B of gp_debug_set knob sets on one library: bash tools/gpu.sh knobab "no_spw=0 no_spw=1" [B K..]
    SETS=$1
    shift
    for rep in 1 2; do
      for S in $SETS; do
        GP_KNOBS=$S run 120 $O/lat_$S.log python -u tools/latency_probe.py ${@:-1048576 20 128}
        echo "== $rep $S"; grep "B=" $O/lat_$S.log
      done
    done ;;
  ab)
    VARS=$1
    shift
    LD=$PWD/gym-po-taxi_amd/gym_po_amd
    for rep in 1 2; do
      for V in $VARS; do
        L=$LD/libgympo_amd_$V.so
        [ "$V" = base ] && L=$LD/libgympo_amd.so
        GYM_PO_AMD_LIB=$L run 120 $O/lat_$V.log python -u tools/latency_probe.py ${@:-1048576 20 128}
        echo "== $rep $V"; grep "B=" $O/lat_$V.log
      done
    done ;;
  copycal)  # FETCH_SIZE / WRITE_SIZE calibration on a 256 MiB device copy (tools/pmc_copy_check.py)
    for P in FETCH_SIZE WRITE_SIZE; do
      run 120 $O/$P.log rocprofv3 --pmc $P --output-format csv -d $O/$P -o p -- python3 tools/pmc_copy_check.py
    done
    python3 tools/pmc_copy_check.py --summarize $O ;;
  measure)  # one call, several lines: the driver-config headline, steady state, crooms, anttag, taxi, VALU costs
    run 300 $O/b_driver.log python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
    last_json $O/b_driver.log 1200
    run 300 $O/b_steady.log python3 bench.py --no-cpu-baseline --steps 1280 --warmup 256 --chunk 128
    last_json $O/b_steady.log 600
    for w in ${MEASURE_WL:-crooms}; do
      run 300 $O/b_$w.log python3 bench.py --no-cpu-baseline --workload $w
      last_json $O/b_$w.log 900
    done
    [ -x tools/mb_valu.bin ] && run 60 $O/mb_valu.txt tools/mb_valu.bin && cat $O/mb_valu.txt
    [ -n "$CRATE" ] && run 300 $O/crooms_rate.jsonl python3 tools/crooms_numpy_rate.py $CRATE && cat $O/crooms_rate.jsonl
    true ;;
  final)  # round-end evidence on the committed build: suite + smoke, rocprof of the driver command, PMC, bench lines
    R=${ROUND:-r03}
    run 1000 $O/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
    tail -n 1 $O/tests.log
    run 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
    run 300 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
    cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/driver_kernel_stats.csv
    i=0
    for C in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      run 300 $O/p$i.log rocprofv3 --pmc $C --output-format csv -d $O/pmc/p$i -o p -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --kernel windowed
      run 300 $O/q$i.log rocprofv3 --pmc $C --output-format csv -d $O/pmcf/p$i -o p -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --kernel fused
    done
    python3 tools/pmc_to_json.py $O/pmc wgrid_rollout fourrooms_hansen4_B1048576_numpy $O/pmc.json fourrooms 20
    cp $O/pmc.json profiles/${R}_pmc_fourrooms_hansen4_B1048576_numpy_K20_wgrid_rollout.json
    python3 tools/pmc_to_json.py $O/pmcf grid_rollout_numpy fourrooms_hansen4_B1048576_numpy $O/pmcf.json fourrooms 20
    cp $O/pmcf.json profiles/${R}_pmc_fourrooms_hansen4_B1048576_numpy_K20_grid_rollout_numpy.json
    run 600 $O/bench_default.log python3 bench.py
    last_json $O/bench_default.log 3000
    run 300 $O/bench_driver.log python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
    last_json $O/bench_driver.log 3000 ;;
  pmcset)  # round-end PMC records beside the driver's: fourrooms at 128 steps per launch, taxi, anttag, crooms
    R=${ROUND:-r03}
    pm() {  # pm <name> <kernel substring> <config key> <workload> <K> <bench args...>
      local n=$1 k=$2 c=$3 w=$4 K=$5
      shift 5
      [ -n "$PMCSET_ONLY" ] && [[ " $PMCSET_ONLY " != *" $w "* ]] && return 0
      local i=0
      for C in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        run 300 $O/$n.p$i.log rocprofv3 --pmc $C --output-format csv -d $O/$n/p$i -o p -- python3 bench.py --no-cpu-baseline "$@"
      done
      python3 tools/pmc_to_json.py $O/$n $k $c $O/$n.json $w $K
      cp $O/$n.json profiles/${R}_pmc_${c}_K${K}_${k}.json
    }
    pm fr128 grid_rollout_numpy fourrooms_hansen4_B1048576_numpy fourrooms 128 --steps 1280 --warmup 256 --chunk 128 --kernel fused
    pm fr128w wgrid_rollout fourrooms_hansen4_B1048576_numpy fourrooms 128 --steps 1280 --warmup 256 --chunk 128 --kernel windowed
    pm taxi taxi_rollout taxi_B4194304_philox taxi 4 --workload taxi
    pm anttag anttag_rollout anttag_B2097152_philox anttag 64 --workload anttag
    pm crooms crooms_rollout crooms_B2097152_philox crooms 128 --workload crooms
    for w in ${PMCSET_ONLY:-taxi anttag crooms}; do
      [ "$w" = fourrooms ] && continue
      run 300 $O/b_$w.log python3 bench.py --no-cpu-baseline --workload $w
      last_json $O/b_$w.log 1500
    done
    [ -n "$PMCSET_ONLY" ] && [[ " $PMCSET_ONLY " != *" fourrooms "* ]] && exit 0
    run 300 $O/b_steady.log python3 bench.py --no-cpu-baseline --steps 1280 --warmup 256 --chunk 128
    last_json $O/b_steady.log 1500 ;;
  micro)  # VALU / PCG64 generation costs and the launch fixed costs (prebuilt tools/*.bin), then the latency probe
    for b in mb_pcg mb_valu mb_lat mb_launch; do
      [ -x tools/$b.bin ] && run 120 $O/$b.txt tools/$b.bin && cat $O/$b.txt
    done
    run 200 $O/lat.log python -u tools/latency_probe.py ${@:-1048576 1 20 128}
    grep "B=" $O/lat.log ;;
  multi)  # 2 ranks share ONE GPU here: the persistent kernels of both must be co-resident (131072 envs each)
    GP_BENCH_BACKEND=gloo run 300 $O/multi2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 256 --warmup 128 --envs 131072 --no-cpu-baseline
    grep '"metric"' $O/multi2.log | cut -c1-900 ;;
  *)
    echo "unknown task '$task'"; exit 2 ;;
esac
echo "GPU_SH_OK $task"
