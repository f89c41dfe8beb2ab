# A/B of an env-var knob on the stamps breakdown and the headline bench: bash tools/gpu_ab.sh VAR "v1 v2 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in $2; do
  echo "== $1=$v"
  env $1=$v timeout -k 10 120 python tools/stamps.py 1048576 > gpurun_out/stamps_$v.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/stamps_$v.log; exit 1; }
  grep -v amdgpu gpurun_out/stamps_$v.log | head -11
  env $1=$v timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/bench_$v.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('value %.3e'%d['value'], 'ms/step %.5f'%d['ms_per_step'])"
done
