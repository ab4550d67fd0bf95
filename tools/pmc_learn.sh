set -e
export TMPDIR=/tmp
D=gpurun_out/pmc_learn
mkdir -p $D
A="--steps 3 --warmup 1 --extra-systems= --update-steps 20 --no-cpu-baseline --no-diagnostics --no-config0 --batches 4096"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_wgrad|k_adam|k_critic|k_actor" -d $D/fetch -o run -- python3 bench.py $A > $D/f.json 2> $D/f.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_wgrad|k_adam|k_critic|k_actor" -d $D/write -o run -- python3 bench.py $A > $D/w.json 2> $D/w.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "k_wgrad|k_adam|k_critic|k_actor" -d $D/sq -o run -- python3 bench.py $A > $D/s.json 2> $D/s.err
python3 tools/prof_summary.py pmc $D/fetch/run_results.db > $D/fetch.csv
python3 tools/prof_summary.py pmc $D/write/run_results.db > $D/write.csv
python3 tools/prof_summary.py pmc $D/sq/run_results.db > $D/sq.csv
