# car_park PER update loop kernel trace (B = 64 and 4096 through the bench's extra systems)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/perprof
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 300 --extra-systems car_park > $D/b.json 2> $D/b.err &&
python3 tools/prof_summary.py stats $D/t/run_results.db > $D/stats.csv &&
python3 tools/timeline.py $D/t/run_results.db k_ 40 200 > $D/timeline.txt &&
rm -rf $D/t
