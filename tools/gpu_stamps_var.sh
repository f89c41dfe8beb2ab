# Stamps breakdown of GP_STAMPS variant libraries (tools/build_variant.sh with BASE=stamps): SVARS="s00 s11"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/svar
mkdir -p $O
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
for V in $SVARS; do
  GYM_PO_AMD_LIB=$LD/libgympo_amd_$V.so timeout -k 10 120 python tools/stamps.py 1048576 ${K:-128} > $O/st_$V.log 2>&1 || { echo STAMPS_FAIL $V; tail -30 $O/st_$V.log; exit 1; }
  echo "== $V"; grep -v amdgpu.ids $O/st_$V.log
done
