set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py 1048576 > gpurun_out/stamps.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/stamps.log | tail -12
timeout -k 10 120 python tools/stamps.py 65536 > gpurun_out/stamps64k.log 2>&1; echo "stamps64k rc=$?"; cat gpurun_out/stamps64k.log | tail -12
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log | cut -c1-900
