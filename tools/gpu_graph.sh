# graph-replay parity test, then the default bench with and without the update graph
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_graph.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-graph --extra-systems "" > gpurun_out/bench_nograph.json 2> gpurun_out/bench_nograph.err
