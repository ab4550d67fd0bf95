# B=4096 update loop under the kernel trace, GEMM variants side by side
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/wg
SMALL="--no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0"
run() {  # name, strips, chunk
  n=$1
  export CACTO_WG_STRIPS=$2 CACTO_WG_CH=$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wg/t_$n -o run -- python3 bench.py --steps 3 --warmup 1 --update-steps 500 --batches 4096 --extra-systems "" $SMALL > gpurun_out/wg/b_$n.json 2> gpurun_out/wg/b_$n.err
  python3 tools/prof_summary.py stats gpurun_out/wg/t_$n/run_results.db > gpurun_out/wg/stats_$n.csv
  python3 tools/prof_gaps.py gpurun_out/wg/t_$n/run_results.db > gpurun_out/wg/gaps_$n.txt 2>&1 || true
  rm -rf gpurun_out/wg/t_$n
}
run old 0 128
run s256 1 256
run s128 1 128
run s512 1 512
