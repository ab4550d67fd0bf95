set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_upd.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python tools/fused_stamps.py > gpurun_out/fstamps.log 2>&1 &&
bash tools/prof_b128.sh > gpurun_out/prof_b128.log 2>&1
