set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_ddp.log 2>&1
