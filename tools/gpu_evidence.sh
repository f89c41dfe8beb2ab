# Round evidence in ONE GPU call: smoke + the -m gpu suite, then for every single-GPU workload the HBM PMC
# passes (FETCH_SIZE / WRITE_SIZE, separate --pmc runs, 128-step launches), the bench line (with CPU
# baseline, picking up the PMC json just written into profiles/), and the rocprofv3 kernel-trace summary.
# Everything lands in gpurun_out/ev/; copy it into profiles/ afterwards.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ev
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
  echo "smoke ok"
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
declare -A KN=([fourrooms]=grid_rollout_numpy [taxi]=taxi_rollout [crooms]=crooms_rollout [anttag]=anttag_rollout)
declare -A CK=([fourrooms]=fourrooms_hansen4_B1048576_numpy [taxi]=taxi_B4194304_philox [crooms]=crooms_B2097152_philox [anttag]=anttag_B2097152_philox)
for W in ${WORKLOADS:-fourrooms taxi crooms anttag}; do
  i=0
  for C in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$W/p$i -o p -- python3 bench.py --workload $W --steps 256 --warmup 128 --no-cpu-baseline > $O/pmc_${W}_p$i.log 2>&1 || { echo "PMC_FAIL $W $C"; tail -20 $O/pmc_${W}_p$i.log; exit 1; }
  done
  python3 tools/pmc_to_json.py $O/pmc_$W ${KN[$W]} ${CK[$W]} $O/r01_pmc_${CK[$W]}.json $W > /dev/null || exit 1
  cp $O/r01_pmc_${CK[$W]}.json profiles/
  timeout -k 10 400 python bench.py --workload $W > $O/bench_$W.log 2>&1 || { echo "BENCH_FAIL $W"; tail -30 $O/bench_$W.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$W.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W', 'value %.4e'%d['value'], 'frac %.3f'%r['frac'], 'traffic', r['traffic'], 'bytes', r['bytes_per_launch'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o bench -- python3 bench.py --workload $W --no-cpu-baseline > $O/prof_$W.log 2>&1 || { echo "PROF_FAIL $W"; tail -20 $O/prof_$W.log; exit 1; }
  for f in $(find $O/prof_$W -name "*kernel_stats.csv"); do cp $f $O/kernel_stats_$W.csv; done
done

# secondary line: FourRooms in rng_mode philox (counter-based draws, no per-step grid exchange)
if [ -z "$SKIP_PHILOX" ]; then
  timeout -k 10 300 python bench.py --mode philox --no-cpu-baseline > $O/bench_fourrooms_philox.log 2>&1 || { echo "BENCH_FAIL philox"; tail -20 $O/bench_fourrooms_philox.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_fourrooms_philox.log').read().strip().splitlines()[-1]); r=d['roofline']; print('fourrooms-philox', 'value %.4e'%d['value'], 'frac %.3f'%r['frac'], r['kernel'])"
fi
echo EVIDENCE_OK
