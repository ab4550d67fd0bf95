# FETCH_SIZE / WRITE_SIZE of the paired q4 chain grid and the fused GEMM + Adam at B = 128 with the
# grid on each given number of XCDs (CACTO_PAIR_XCDS). Usage: bash tools/pmc_xmap.sh 8 4 2
set -e
export TMPDIR=/tmp
D=gpurun_out/pmc_xmap
mkdir -p $D
A="--steps 3 --warmup 1 --extra-systems= --update-steps 20 --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 --batches 128"
for X in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    CACTO_PAIR_XCDS=$X timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_chain_pair|k_wgrad_adam" -d $D/x$X$C -o run -- python3 bench.py $A > $D/x$X$C.json 2> $D/x$X$C.err
    python3 tools/prof_summary.py pmc $D/x$X$C/run_results.db > $D/x${X}_$C.csv
    rm -rf $D/x$X$C
  done
done
