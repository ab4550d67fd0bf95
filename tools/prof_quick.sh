# Kernel-trace summary of one bench invocation: bash tools/prof_quick.sh NAME [bench args...]
set -e
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/pq
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/pq/$name -o run -- python3 bench.py --no-cpu-baseline --no-diagnostics "$@" > gpurun_out/pq/$name.json 2> gpurun_out/pq/$name.err
python3 tools/prof_summary.py stats gpurun_out/pq/$name/run_results.db > gpurun_out/pq/$name.csv
