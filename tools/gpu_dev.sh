# Development GPU call: selected -m gpu tests (TESTS, default all), then one bench line per workload in
# BENCHES (default none), optionally a rocprofv3 kernel-trace summary of each (PROF=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dev
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS}" ] || [ -z "${BENCHES}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -40; tail -60 $O/tests.log; exit 1; }
  grep -cE "PASSED" $O/tests.log; tail -2 $O/tests.log
fi
for W in ${BENCHES}; do
  timeout -k 10 300 python bench.py --workload $W ${BENCH_ARGS} > $O/bench_$W.log 2>&1 || { echo "BENCH_FAIL $W"; tail -30 $O/bench_$W.log; exit 1; }
  tail -1 $O/bench_$W.log
  if [ -n "${PROF}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o bench -- python3 bench.py --workload $W --no-cpu-baseline ${BENCH_ARGS} > $O/prof_$W.log 2>&1 || { echo "PROF_FAIL $W"; tail -20 $O/prof_$W.log; exit 1; }
    for f in $(find $O/prof_$W -name "*kernel_stats.csv"); do cp $f $O/kernel_stats_$W.csv; head -4 $f | cut -c1-300; done
  fi
done
echo DEV_OK
