# Kernel trace of the DI update loop at batch B (default 4096) and the gaps between consecutive
# weight-gradient launches. Usage: bash tools/prof_update.sh [B]
set -e
export TMPDIR=/tmp
B=${1:-4096}
D=gpurun_out/prof_b$B
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run -- python3 bench.py --steps 5 --warmup 2 --update-steps 500 --batches $B --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 > $D/b.json 2> $D/b.err
python3 tools/prof_summary.py stats $D/t/run_results.db > $D/stats.csv
python3 tools/timeline.py $D/t/run_results.db k_ 40 200 > $D/timeline.txt
rm -rf $D/t
