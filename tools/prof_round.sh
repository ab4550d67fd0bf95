# Round profile set (see profiles/README.md). Usage: bash tools/prof_round.sh r06
#  1. kernel trace of the default bench (every system), and of the DI update loop at B = 128 and at
#     B = 4096 in runs of their own (so per-batch learner kernel times are readable);
#  2. PMC passes, one counter group per run (TCC slot limits): FETCH_SIZE, WRITE_SIZE and MFMA busy /
#     MOPS / GRBM_GUI_ACTIVE of the rollout kernels of DI (4096), the manipulator (8192) and UR5
#     (2048); MFMA counters and FETCH_SIZE / WRITE_SIZE of the learner kernels at B = 128 and 4096 (DI).
#  Counter collection serializes kernels: the update pipeline's one-time concurrency probe then
#  orders its streams with queue markers by itself (bench.py's "update_pipeline" records which).
set -e
export TMPDIR=/tmp
R=$1
D=gpurun_out/prof_$R
mkdir -p $D
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --no-dp1 --long-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 200 $SMALL > $D/bench_under_rocprof.json 2> $D/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b128 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 128 --extra-systems "" $SMALL > $D/b128.json 2> $D/b128.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/b4096 -o run -- python3 bench.py --steps 10 --warmup 2 --update-steps 1000 --batches 4096 --extra-systems "" $SMALL > $D/b4096.json 2> $D/b4096.err
python3 tools/prof_summary.py stats $D/trace/run_results.db > $D/kernel_stats.csv
python3 tools/prof_summary.py stats $D/b128/run_results.db > $D/kernel_stats_di_b128.csv
python3 tools/prof_summary.py stats $D/b4096/run_results.db > $D/kernel_stats_di_b4096.csv
rm -rf $D/trace $D/b128 $D/b4096
PMCARGS="--steps 3 --warmup 1 --extra-systems= --update-steps 20 $SMALL"
MFMA="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for S in double_integrator:4096 manipulator:8192 ur5:2048; do
  sys=${S%%:*}; n=${S##*:}
  ROLL="--system $sys --rollouts $n --batches 128"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rollout -d $D/fetch_$sys -o run -- python3 bench.py $PMCARGS $ROLL > $D/fetch_$sys.json 2> $D/fetch_$sys.err
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_rollout -d $D/write_$sys -o run -- python3 bench.py $PMCARGS $ROLL > $D/write_$sys.json 2> $D/write_$sys.err
  timeout -s KILL 120 rocprofv3 --pmc $MFMA --kernel-include-regex k_rollout -d $D/mfma_$sys -o run -- python3 bench.py $PMCARGS $ROLL > $D/mfma_$sys.json 2> $D/mfma_$sys.err
  python3 tools/prof_summary.py pmc $D/fetch_$sys/run_results.db > $D/pmc_fetch_$sys.csv
  python3 tools/prof_summary.py pmc $D/write_$sys/run_results.db > $D/pmc_write_$sys.csv
  python3 tools/prof_summary.py pmc $D/mfma_$sys/run_results.db > $D/pmc_mfma_rollout_$sys.csv
  rm -rf $D/fetch_$sys $D/write_$sys $D/mfma_$sys
done
LEARN="k_chain_pair|k_critic_grad|k_actor_grad|k_wgrad|k_adam"
for B in 128 4096; do
  timeout -s KILL 120 rocprofv3 --pmc $MFMA --kernel-include-regex "$LEARN" -d $D/mfma$B -o run -- python3 bench.py $PMCARGS --batches $B > $D/mfma$B.json 2> $D/mfma$B.err
  python3 tools/prof_summary.py pmc $D/mfma$B/run_results.db > $D/pmc_mfma_b$B.csv
  rm -rf $D/mfma$B
  for C in FETCH_SIZE WRITE_SIZE; do
    c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$LEARN" -d $D/l${c}$B -o run -- python3 bench.py $PMCARGS --batches $B > $D/l${c}$B.json 2> $D/l${c}$B.err
    python3 tools/prof_summary.py pmc $D/l${c}$B/run_results.db > $D/pmc_learn_${c}_b$B.csv
    rm -rf $D/l${c}$B
  done
done
