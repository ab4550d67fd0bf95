# learner iteration: update parity / pipeline tests, then the bench (no CPU legs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_main_loop.py tests/test_gpu_dp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_upd.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config0 > gpurun_out/bench_upd.json 2> gpurun_out/bench_upd.err
