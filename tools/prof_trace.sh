set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-diagnostics > gpurun_out/prof/bench_under_rocprof.json 2> gpurun_out/prof/trace.err
python3 tools/prof_summary.py stats gpurun_out/prof/trace/run_results.db > gpurun_out/prof/kernel_stats.csv
