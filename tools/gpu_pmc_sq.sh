# SQ counter passes (VALU / LDS / waits per wave, busy cycles) for one workload's rollout kernel.
#   W=anttag K=anttag_rollout bash tools/gpu_pmc_sq.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmcsq_$W
mkdir -p $O
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p -- python3 bench.py --workload $W --steps 256 --warmup 128 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O $K
