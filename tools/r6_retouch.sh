# Round 6: bench.py's driver command with and without re-touching the output buffers after the warmup
# (GP_BENCH_NO_RETOUCH=1 skips it), three alternating runs each; one GPU step at a time, the first failure ends.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rt
for i in 1 2 3; do
  for v in 0 1; do
    if [ $v = 1 ]; then export GP_BENCH_NO_RETOUCH=1; else unset GP_BENCH_NO_RETOUCH; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/rt/run_${i}_${v}.log 2>&1 || exit 1
    echo "no_retouch=$v $(tail -n1 gpurun_out/rt/run_${i}_${v}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"])')"
  done
done
