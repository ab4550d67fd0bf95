# FETCH_SIZE of k_wgrad at DI B = 4096 with the chunks grouped by XCD (CACTO_WG_XCD=1) and not (0).
set -e
export TMPDIR=/tmp
D=gpurun_out/pmc_wgrad
mkdir -p $D
A="--steps 3 --warmup 1 --extra-systems= --update-steps 20 --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 --batches 4096"
for X in 0 1; do
  CACTO_WG_XCD=$X timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_wgrad|k_adam" -d $D/x$X -o run -- python3 bench.py $A > $D/x$X.json 2> $D/x$X.err
  python3 tools/prof_summary.py pmc $D/x$X/run_results.db > $D/x${X}_fetch.csv
  rm -rf $D/x$X
done
