set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ws gpurun_out/t6
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgrid_gpu.py tests/test_bench_path_gpu.py -m gpu > gpurun_out/t6/tests.log 2>&1 || { tail -40 gpurun_out/t6/tests.log; exit 1; }
tail -2 gpurun_out/t6/tests.log
bash tools/gpu.sh knobab "wg_tmode=0 wg_tmode=2048" 1048576 20 128
GYM_PO_AMD_LIB=$PWD/gym-po-taxi_amd/gym_po_amd/libgympo_amd_r4.so timeout -k 10 120 python -u tools/latency_probe.py 1048576 20 128 | grep B=
WSTAMPS_RAW=gpurun_out/ws/raw0.npz timeout -k 10 120 python -u tools/wstamps.py 1048576 64 > gpurun_out/ws/t0.txt 2>&1
