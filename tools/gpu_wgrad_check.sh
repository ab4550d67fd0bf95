set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_upd.log 2>&1 &&
bash tools/prof_b4096.sh > gpurun_out/prof_b4096.log 2>&1
