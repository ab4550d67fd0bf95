# learner PMC passes again with queue-marker ordering (the device-side waits spin under counter
# collection's serialization), into gpurun_out/prof_r05t
set -e
export TMPDIR=/tmp
export CACTO_PIPE_DEVWAIT=0
D=gpurun_out/prof_r05t
mkdir -p $D
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0"
PMCARGS="--steps 3 --warmup 1 --extra-systems= --update-steps 20 $SMALL"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_rollout|k_critic_grad|k_actor_grad|k_wgrad|k_chain_pair" -d $D/mfma4096 -o run -- python3 bench.py $PMCARGS --batches 4096 > $D/mfma4096.json 2> $D/mfma4096.err
python3 tools/prof_summary.py pmc $D/mfma4096/run_results.db > $D/pmc_mfma_b4096.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_rollout|k_critic_grad|k_actor_grad|k_wgrad|k_chain_pair" -d $D/mfma128 -o run -- python3 bench.py $PMCARGS --batches 128 > $D/mfma128.json 2> $D/mfma128.err
python3 tools/prof_summary.py pmc $D/mfma128/run_results.db > $D/pmc_mfma_b128.csv
LEARN="k_chain_pair|k_critic_grad|k_actor_grad|k_wgrad|k_adam"
for B in 128 4096; do
  for C in FETCH_SIZE WRITE_SIZE; do
    c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$LEARN" -d $D/l${c}$B -o run -- python3 bench.py $PMCARGS --batches $B > $D/l${c}$B.json 2> $D/l${c}$B.err
    python3 tools/prof_summary.py pmc $D/l${c}$B/run_results.db > $D/pmc_learn_${c}_b$B.csv
  done
done
for d in mfma128 mfma4096 lfetch128 lwrite128 lfetch4096 lwrite4096; do rm -rf $D/$d; done
cat $D/pmc_learn_fetch_b4096.csv $D/pmc_learn_write_b4096.csv
