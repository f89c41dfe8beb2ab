# Performance investigation helper: batch-size sweep + PMC counter passes on the step kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
for B in 65536 1048576 4194304; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --envs $B --no-cpu-baseline > gpurun_out/sweep_$B.log 2>&1 || { echo "sweep $B failed"; tail -5 gpurun_out/sweep_$B.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$B.log').read().strip().splitlines()[-1]); print($B, 'ms/step %.4f'%d['ms_per_step'], 'kernel_us %.2f'%d['roofline']['kernel_avg_us'], 'GB/s %.0f'%d['roofline']['achieved'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
         "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc/p$i -o p -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc grid_step_numpy grid_resolve_numpy
