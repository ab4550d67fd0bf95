# kernel traces of the final bench (the first part of prof_round.sh) into gpurun_out/prof_r05c
set -e
export TMPDIR=/tmp
D=gpurun_out/prof_r05c
mkdir -p $D
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 200 --no-cpu-baseline --no-diagnostics --no-config0 > $D/bench_under_rocprof.json 2> $D/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b128 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 128 --extra-systems "" $SMALL > $D/b128.json 2> $D/b128.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b4096 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 4096 --extra-systems "" $SMALL > $D/b4096.json 2> $D/b4096.err
python3 tools/prof_summary.py stats $D/trace/run_results.db > $D/kernel_stats.csv
python3 tools/prof_summary.py stats $D/b128/run_results.db > $D/kernel_stats_di_b128.csv
python3 tools/prof_summary.py stats $D/b4096/run_results.db > $D/kernel_stats_di_b4096.csv
python3 tools/timeline.py $D/b4096/run_results.db k_ 40 200 > $D/timeline_di_b4096.txt
for d in trace b128 b4096; do rm -rf $D/$d; done
grep -E "k_rollout_ks<2>|k_critic_grad,|k_actor_grad<2>|k_wgrad_big|k_chain_pair_q4<2>|k_wgrad_adam" $D/kernel_stats.csv
