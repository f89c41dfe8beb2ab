set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --mode philox --no-cpu-baseline > gpurun_out/bench_philox.log 2>&1; echo "bench philox rc=$?"; tail -1 gpurun_out/bench_philox.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o fr -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"
find gpurun_out/prof -name "*stats*" | head; for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do head -8 $f; done
