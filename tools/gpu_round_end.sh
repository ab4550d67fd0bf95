# everything the driver runs at round end, in one call: GPU tests, smoke(), the default bench line,
# then the round's rocprofv3 profile set. Usage: bash tools/gpu_round_end.sh r02
set -o pipefail
export TMPDIR=/tmp
R=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err &&
bash tools/prof_round.sh $R
