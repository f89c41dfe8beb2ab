set -e
export TMPDIR=/tmp
bash tools/gpu.sh knobab "wg_tmode=0 wg_tmode=128 wg_tmode=2176 wg_tmode=384 wg_tmode=192 wg_tmode=32 wg_tmode=4224 wg_tmode=256" 1048576 20 128
GP_KNOBS=wg_tmode=128 timeout -k 10 120 python -u tools/wstamps.py 1048576 64 > gpurun_out/ws/t128.txt 2>&1
