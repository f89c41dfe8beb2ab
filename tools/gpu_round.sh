# One GPU call: smoke, -m gpu tests, the default bench line, the rocprof kernel-trace summary of the
# bench command, and FETCH_SIZE / WRITE_SIZE passes (separate --pmc runs). Everything lands in
# gpurun_out/round/; copy what is judged into profiles/ afterwards.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/round
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
echo "smoke ok"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests/ -x -q -m gpu ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
for f in $(find $O/prof -name "*kernel_stats.csv"); do cp $f $O/kernel_stats.csv; head -6 $f; done
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc/p$i -o p -- python3 bench.py --steps 256 --warmup 64 --no-cpu-baseline ${BENCH_ARGS} > $O/pmc_p$i.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $O/pmc_p$i.log; exit 1; }
done
python3 tools/pmc_to_json.py $O/pmc ${PMC_KERNEL:-grid_rollout_numpy} ${PMC_CFG:-fourrooms_hansen4_B1048576_numpy} $O/pmc.json ${PMC_WORKLOAD:-fourrooms}
echo ROUND_OK
