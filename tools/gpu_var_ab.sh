# In-call A/B of library variants (latency probe at K = 1 and 128, kernel-event time per launch).
#   VARS="ab v_top_val ..." bash tools/gpu_var_ab.sh   (ab = libgympo_amd_ab.so, "" = libgympo_amd.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/var
mkdir -p $O
LD=$GRAFT_REPO_ROOT/gym-po-taxi_amd/gym_po_amd
for rep in 1 2; do
  for V in $VARS; do
    L=libgympo_amd_$V.so
    GYM_PO_AMD_LIB=$LD/$L timeout -k 10 120 python -u tools/latency_probe.py 1048576 ${KS:-1 128} > $O/lat_$V.log 2>&1 || { echo LAT_FAIL $V; tail -20 $O/lat_$V.log; exit 1; }
    echo "== $rep $V"; grep "B=" $O/lat_$V.log | sed 's/host wall median/wall/; s/(p10 [0-9.]*); //'
  done
done
