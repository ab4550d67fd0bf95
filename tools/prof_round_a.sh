# round profile set, part A (see tools/prof_round.sh): GPU tests, smoke, the default bench line,
# kernel traces (default bench, DI B = 128, DI B = 4096). Usage: bash tools/prof_round_a.sh r03
set -o pipefail
export TMPDIR=/tmp
R=$1
D=gpurun_out/prof_$R
mkdir -p $D
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/gpu_all.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_full.json 2> $D/bench_full.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 200 $SMALL > $D/bench_under_rocprof.json 2> $D/trace.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/b128 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 128 --extra-systems "" $SMALL > $D/b128.json 2> $D/b128.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/b4096 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 4096 --extra-systems "" $SMALL > $D/b4096.json 2> $D/b4096.err &&
python3 tools/prof_summary.py stats $D/trace/run_results.db > $D/kernel_stats.csv &&
python3 tools/prof_summary.py stats $D/b128/run_results.db > $D/kernel_stats_di_b128.csv &&
python3 tools/prof_summary.py stats $D/b4096/run_results.db > $D/kernel_stats_di_b4096.csv &&
python3 tools/timeline.py $D/b4096/run_results.db k_ 24 400 > $D/timeline_b4096.txt &&
rm -rf $D/trace $D/b128 $D/b4096
