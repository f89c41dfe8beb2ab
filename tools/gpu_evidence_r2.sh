# Round 2 evidence in ONE GPU call (everything under gpurun_out/ev2/; copy into profiles/ afterwards):
#  1. HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate --pmc runs) for every workload at its bench launch
#     shape, and for the headline also at the driver's K = 20 -> profiles/r02_pmc_*.json (bench.py reads them);
#  2. SQ instruction / busy counters of the headline kernel (2 passes);
#  3. bench lines: headline at the driver config (--steps 20 --warmup 5, with CPU baseline) and steady state
#     (--steps 2000), the other workloads at their defaults (with CPU baselines);
#  4. rocprofv3 --kernel-trace --stats of the headline at both shapes.
# FR_ONLY=1: only the headline (FourRooms) parts, after a change to its kernel alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ev2
mkdir -p $O
export TMPDIR=/tmp
declare -A KN=([fourrooms]=grid_rollout_numpy [taxi]=taxi_rollout [crooms]=crooms_rollout [anttag]=anttag_rollout)
declare -A CK=([fourrooms]=fourrooms_hansen4_B1048576_numpy [taxi]=taxi_B4194304_philox [crooms]=crooms_B2097152_philox [anttag]=anttag_B2097152_philox)
declare -A CH=([fourrooms]=128 [taxi]=4 [crooms]=128 [anttag]=64)
pmc() {  # workload chunk steps warmup tag
  local W=$1 C=$2 S=$3 WU=$4 T=$5 i=0
  for P in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$T/p$i -o p -- python3 bench.py --workload $W --chunk $C --steps $S --warmup $WU --no-cpu-baseline > $O/pmc_${T}_p$i.log 2>&1 || { echo "PMC_FAIL $T $P"; tail -20 $O/pmc_${T}_p$i.log; return 1; }
  done
  python3 tools/pmc_to_json.py $O/pmc_$T ${KN[$W]} ${CK[$W]} $O/r02_pmc_${CK[$W]}_K$C.json $W $C && cp $O/r02_pmc_${CK[$W]}_K$C.json profiles/
}
pmc fourrooms 128 256 128 fr128 || exit 1
pmc fourrooms 20 200 100 fr20 || exit 1
if [ -z "$FR_ONLY" ]; then for W in taxi crooms anttag; do pmc $W ${CH[$W]} 256 128 $W || exit 1; done; fi
echo PMC_OK
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/sq/p$i -o p -- python3 bench.py --steps 256 --warmup 128 --no-cpu-baseline > $O/sq_p$i.log 2>&1 || { echo "SQ pass $i failed"; tail -5 $O/sq_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/sq grid_rollout_numpy grid_rollout_counter > $O/sq_summary.txt 2>&1 || true
echo SQ_OK
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_fourrooms_driver.log 2>&1 || { echo BENCH_FAIL driver; tail -30 $O/bench_fourrooms_driver.log; exit 1; }
tail -n 1 $O/bench_fourrooms_driver.log | cut -c 1-400
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_fourrooms_steady.log 2>&1 || { echo BENCH_FAIL steady; tail -30 $O/bench_fourrooms_steady.log; exit 1; }
if [ -z "$FR_ONLY" ]; then for W in taxi crooms anttag; do
  timeout -k 10 400 python bench.py --workload $W > $O/bench_$W.log 2>&1 || { echo "BENCH_FAIL $W"; tail -30 $O/bench_$W.log; exit 1; }
done; fi
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f'.split('/')[-1], 'value %.4e'%d['value'], 'ms/step %.5f'%d['ms_per_step'], 'frac %.3f'%r['frac'], 'traffic/alg', r.get('traffic_over_algorithmic'))"; done
echo BENCH_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_driver.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_driver.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_steady -o bench -- python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/prof_steady.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_steady.log; exit 1; }
for t in driver steady; do for f in $(find $O/prof_$t -name "*kernel_stats.csv"); do cp $f $O/kernel_stats_fourrooms_$t.csv; done; done
echo EVIDENCE_OK
