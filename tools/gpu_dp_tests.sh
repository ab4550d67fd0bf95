set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dp.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_dp.log 2>&1
