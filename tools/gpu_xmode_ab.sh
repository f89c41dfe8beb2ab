# Stamps A/B of GP_XMODE settings (stamps build): e.g. XMS="1 5" (5 = no output stores: hop latency without
# the output write stream).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/xab
mkdir -p $O
for rep in 1 2; do
for x in ${XMS:-1 5}; do
  GP_XMODE=$x timeout -k 10 120 python tools/stamps.py 1048576 ${K:-128} > $O/st_$x.log 2>&1 || { echo STAMPS_FAIL; tail -30 $O/st_$x.log; exit 1; }
  echo "== $rep GP_XMODE=$x"; grep -v amdgpu.ids $O/st_$x.log | grep -E "event-timed|transitions|B1 wait|exchange done|resets|advance|step \(|publish|poll done|gather done|draw cells|staging written|B2 wait"
done
done
