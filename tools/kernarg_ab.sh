# In-call A/B of the kernel-argument placement (HIP_FORCE_DEV_KERNARG 1 = device memory, 0 = runtime default)
# around the driver-shaped launch: host wall and event-timed kernel per call (tools/latency_probe.py).
set -eo pipefail
mkdir -p gpurun_out/kab
for rep in 1 2; do
  for v in 1 0; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python -u tools/latency_probe.py ${@:-1048576 20 128} > gpurun_out/kab/k$v.log 2>&1
    echo "== $rep dev_kernarg=$v"; grep "B=" gpurun_out/kab/k$v.log
  done
done
