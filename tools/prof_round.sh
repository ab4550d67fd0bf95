# Round profile set (see profiles/README.md). Usage: bash tools/prof_round.sh r03
#  1. kernel trace of the default bench (every system), and of the DI update loop at B = 128 and at
#     B = 4096 in runs of their own (so per-batch learner kernel times are readable);
#  2. PMC passes, one counter group per run (TCC slot limits): FETCH_SIZE, WRITE_SIZE of the
#     rollout; MFMA busy cycles / MFMA MOPS / GRBM_GUI_ACTIVE of the rollout and learner kernels;
#     FETCH_SIZE, WRITE_SIZE of the learner kernels at B = 128 and B = 4096 (DI only).
set -e
export TMPDIR=/tmp
R=$1
D=gpurun_out/prof_$R
mkdir -p $D
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 200 $SMALL > $D/bench_under_rocprof.json 2> $D/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b128 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 128 --extra-systems "" $SMALL > $D/b128.json 2> $D/b128.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b4096 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 4096 --extra-systems "" $SMALL > $D/b4096.json 2> $D/b4096.err
PMCARGS="--steps 3 --warmup 1 --extra-systems= --update-steps 20 $SMALL"
# counter collection serializes the kernels: the two-stream pipeline's device-side waits would then
# hold the queue their producer needs, so the PMC passes order the streams with queue markers
export CACTO_PIPE_DEVWAIT=0
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rollout -d $D/fetch -o run -- python3 bench.py $PMCARGS --batches 128 > $D/fetch.json 2> $D/fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_rollout -d $D/write -o run -- python3 bench.py $PMCARGS --batches 128 > $D/write.json 2> $D/write.err
python3 tools/prof_summary.py stats $D/trace/run_results.db > $D/kernel_stats.csv
python3 tools/prof_summary.py stats $D/b128/run_results.db > $D/kernel_stats_di_b128.csv
python3 tools/prof_summary.py stats $D/b4096/run_results.db > $D/kernel_stats_di_b4096.csv
python3 tools/prof_summary.py pmc $D/fetch/run_results.db > $D/pmc_fetch.csv
python3 tools/prof_summary.py pmc $D/write/run_results.db > $D/pmc_write.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_rollout|k_critic_grad|k_actor_grad|k_wgrad|k_chain_pair" -d $D/mfma128 -o run -- python3 bench.py $PMCARGS --batches 128 > $D/mfma128.json 2> $D/mfma128.err
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_rollout|k_critic_grad|k_actor_grad|k_wgrad|k_chain_pair" -d $D/mfma4096 -o run -- python3 bench.py $PMCARGS --batches 4096 > $D/mfma4096.json 2> $D/mfma4096.err
python3 tools/prof_summary.py pmc $D/mfma128/run_results.db > $D/pmc_mfma_b128.csv
python3 tools/prof_summary.py pmc $D/mfma4096/run_results.db > $D/pmc_mfma_b4096.csv
LEARN="k_chain_pair|k_critic_grad|k_actor_grad|k_wgrad|k_adam"
for B in 128 4096; do
  for C in FETCH_SIZE WRITE_SIZE; do
    c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$LEARN" -d $D/l${c}$B -o run -- python3 bench.py $PMCARGS --batches $B > $D/l${c}$B.json 2> $D/l${c}$B.err
    python3 tools/prof_summary.py pmc $D/l${c}$B/run_results.db > $D/pmc_learn_${c}_b$B.csv
  done
done
# keep the summaries only (the raw rocprofv3 databases would overflow the copy-back)
for d in trace b128 b4096 fetch write mfma128 mfma4096 lfetch128 lwrite128 lfetch4096 lwrite4096; do rm -rf $D/$d; done
