set -e
mkdir -p gpurun_out/ws
for T in 0 2; do
GP_KNOBS=wg_tmode=$T WSTAMPS_RAW=gpurun_out/ws/raw$T.npz timeout -k 10 120 python -u tools/wstamps.py 1048576 64 > gpurun_out/ws/t$T.txt 2>&1
done
timeout -k 10 120 python -u tools/latency_probe.py 1048576 20 128 | grep B=
