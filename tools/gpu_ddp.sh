# DDP parity + .h5 GPU tests, then a short bench pass reporting the DDP label timings of every system
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py tests/test_h5.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_ddp.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diagnostics --batches 128 --update-steps 5 > gpurun_out/bench_ddp.json 2> gpurun_out/bench_ddp.err
