# Stamps of the early-count kernel vs the B1 kernel, and the early kernel without output stores (GP_XMODE=5).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/svar
mkdir -p $O
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
run() {  # name lib xmode
  GP_XMODE=$3 GYM_PO_AMD_LIB=$LD/libgympo_amd_$2.so timeout -k 10 120 python tools/stamps.py 1048576 128 > $O/st_$1.log 2>&1 || { echo STAMPS_FAIL $1; tail -30 $O/st_$1.log; exit 1; }
  echo "== $1"; grep -v amdgpu.ids $O/st_$1.log
}
for v in ${SV:-se0 se1}; do run $v $v 1 || exit 1; done
