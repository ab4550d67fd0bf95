# Round profile set (see profiles/README.md): kernel trace of the default bench, then FETCH_SIZE and
# WRITE_SIZE of k_rollout in separate passes. Usage: bash tools/prof_round.sh r01
set -e
export TMPDIR=/tmp
R=$1
D=gpurun_out/prof_$R
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-diagnostics > $D/bench_under_rocprof.json 2> $D/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rollout -d $D/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diagnostics --extra-systems "" --batches 128 --update-steps 5 > $D/fetch.json 2> $D/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_rollout -d $D/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diagnostics --extra-systems "" --batches 128 --update-steps 5 > $D/write.json 2> $D/write.err
python3 tools/prof_summary.py stats $D/trace/run_results.db > $D/kernel_stats.csv
python3 tools/prof_summary.py pmc $D/fetch/run_results.db > $D/pmc_fetch.csv
python3 tools/prof_summary.py pmc $D/write/run_results.db > $D/pmc_write.csv
