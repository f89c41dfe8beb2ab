# Taxi (configs[2]) PMC traffic + bench line after a change to taxi.hip (outputs under gpurun_out/ev2/).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ev2
mkdir -p $O
export TMPDIR=/tmp
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_taxi/p$i -o p -- python3 bench.py --workload taxi --chunk 4 --steps 256 --warmup 128 --no-cpu-baseline > $O/pmc_taxi_p$i.log 2>&1 || { echo "PMC_FAIL $P"; tail -20 $O/pmc_taxi_p$i.log; exit 1; }
done
python3 tools/pmc_to_json.py $O/pmc_taxi taxi_rollout taxi_B4194304_philox $O/r02_pmc_taxi_B4194304_philox_K4.json taxi 4 || exit 1
cp $O/r02_pmc_taxi_B4194304_philox_K4.json profiles/
timeout -k 10 400 python bench.py --workload taxi > $O/bench_taxi.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_taxi.log; exit 1; }
tail -n 1 $O/bench_taxi.log | cut -c 1-300
