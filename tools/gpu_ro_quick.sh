# rollout iteration without stamps: rollout parity / full-size tests, then the bench (no CPU legs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_main_loop.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_ro.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config0 > gpurun_out/bench_ro.json 2> gpurun_out/bench_ro.err
