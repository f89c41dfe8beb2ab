# A/B inside one call: kernel-argument placement (HIP_FORCE_DEV_KERNARG) vs the fused launch's prologue.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/kab
mkdir -p $O
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python tools/stamps.py 1048576 20 > $O/st_$v.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/st_$v.log; exit 1; }
  echo "== HIP_FORCE_DEV_KERNARG=$v"; grep -v amdgpu.ids $O/st_$v.log | head -4
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python -u tools/latency_probe.py 1048576 1 20 > $O/lat_$v.log 2>&1 || { echo LAT_FAIL; tail -20 $O/lat_$v.log; exit 1; }
  grep "B=" $O/lat_$v.log
done
