# Host launch+sync overhead of the fused rollout under different host wait policies.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lat
mkdir -p $O
timeout -k 10 180 python -u tools/latency_probe.py 1048576 1 20 128 > $O/default.log 2>&1 || { echo FAIL_default; tail -20 $O/default.log; exit 1; }
cat $O/default.log
ROC_ACTIVE_WAIT_TIMEOUT=1000000 timeout -k 10 180 python -u tools/latency_probe.py 1048576 1 20 128 > $O/awt.log 2>&1 || { echo FAIL_awt; tail -20 $O/awt.log; exit 1; }
echo "== ROC_ACTIVE_WAIT_TIMEOUT=1000000"; cat $O/awt.log
timeout -k 10 180 python -u tools/latency_probe.py --spin early 1048576 1 20 128 > $O/spin_early.log 2>&1 || { echo FAIL_spin_early; tail -20 $O/spin_early.log; exit 1; }
echo "== spin early"; cat $O/spin_early.log
timeout -k 10 180 python -u tools/latency_probe.py --spin late 1048576 1 20 128 > $O/spin_late.log 2>&1 || { echo FAIL_spin_late; tail -20 $O/spin_late.log; exit 1; }
echo "== spin late"; cat $O/spin_late.log
