# In-call A/B of C-ROOMS exact-mode throughput across library variants: bash tools/crooms_ab.sh "base r03 v1" [B]
set -eo pipefail
mkdir -p gpurun_out/crab
LD=$PWD/gym-po-taxi_amd/gym_po_amd
for rep in 1 2; do
  for V in $1; do
    L=$LD/libgympo_amd_$V.so
    [ "$V" = base ] && L=$LD/libgympo_amd.so
    GYM_PO_AMD_LIB=$L timeout -k 10 200 python -u tools/crooms_numpy_rate.py ${2:-65536} > gpurun_out/crab/$V.log 2>&1
    echo "== $rep $V"; grep '"numpy"' gpurun_out/crab/$V.log
  done
done
