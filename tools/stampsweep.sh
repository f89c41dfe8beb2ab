mkdir -p gpurun_out/ws7
for T in ${TMODES:-0 64}; do
  GP_KNOBS=wg_tmode=$T timeout -k 10 120 python -u tools/wstamps.py 1048576 64 > gpurun_out/ws7/t$T.txt 2>&1 || { echo FAIL $T; tail -5 gpurun_out/ws7/t$T.txt; exit 1; }
  echo "== tmode $T"; grep -E "event-timed|step \(|env:|ctrl:|spread|last publish|store:" gpurun_out/ws7/t$T.txt
done
