# PMC passes on the headline bench (fused numpy rollout kernel, 64 steps per launch).
# Separate --pmc passes, kernel-trace/stats only (no sys/runtime traces with --pmc).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA" \
         "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc/p$i -o p -- python3 bench.py --steps 256 --warmup 128 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc grid_rollout_numpy grid_rollout_counter
