# everything the driver runs at round end, in one call: GPU tests, smoke(), the default bench line,
# then the round's rocprofv3 profile set
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err &&
bash tools/prof_round.sh r01
