# Full -m gpu suite + smoke on the current build (round-end gate).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ta
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
