set -e
export TMPDIR=/tmp
O=gpurun_out/m2; mkdir -p $O
bash tools/gpu.sh hiptrace --steps 20 --warmup 5
python3 tools/host_gap.py gpurun_out/hiptrace/out > $O/host_gap.txt 2>&1 || true
for B in 131072 262144; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --envs $B --steps 1280 --warmup 256 > $O/strong_$B.log 2>&1
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --envs $B --steps 20 --warmup 5 > $O/strong20_$B.log 2>&1
done
SQ_KERNELS=crooms_rollout bash tools/gpu.sh sq --workload crooms --steps 256 --warmup 128
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xg -o p -- python3 tools/crooms_numpy_rate.py 65536 > $O/xg.log 2>&1
echo M2_OK
