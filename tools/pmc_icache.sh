# instruction-cache counters of the learner kernels at B = 128 (paired pipeline) and 4096
set -e
export TMPDIR=/tmp
D=gpurun_out/pmc_icache
mkdir -p $D
A="--steps 3 --warmup 1 --extra-systems= --update-steps 20 --no-cpu-baseline --no-diagnostics --no-config0"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_wgrad|k_chain|k_critic|k_actor|k_rollout<2" -d $D/p -o run -- python3 bench.py $A --batches 128,4096 > $D/p.json 2> $D/p.err
python3 tools/prof_summary.py pmc $D/p/run_results.db > $D/icache.csv
