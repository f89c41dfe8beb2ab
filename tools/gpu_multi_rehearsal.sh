# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks (gloo, both on cuda:0) under torch.distributed.run.
# The real multi-GPU runs use one rank per GPU over RCCL (the driver's 8-GPU node).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 256 --warmup 128 --envs 262144 \
  --no-cpu-baseline > gpurun_out/multi2.log 2>&1 || { echo MULTI_FAIL; tail -30 gpurun_out/multi2.log; exit 1; }
grep '"metric"' gpurun_out/multi2.log | cut -c1-700
