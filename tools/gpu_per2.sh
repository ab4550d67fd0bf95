# PER multi-workgroup kernels: parity tests (default and forced), car_park rates, kernel trace
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/per2
mkdir -p $D
T="tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py tests/test_gpu_main_loop.py tests/test_gpu_graph.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
CACTO_PER_MW_MIN=1 timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread -k "per or PER or Per or buffer or main_loop" > $D/tests_mw1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 500 --extra-systems car_park > $D/bplain.json 2> $D/bplain.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 300 --extra-systems car_park > $D/b.json 2> $D/b.err &&
python3 tools/prof_summary.py stats $D/t/run_results.db > $D/stats.csv &&
python3 tools/timeline.py $D/t/run_results.db k_ 30 200 > $D/timeline.txt &&
rm -rf $D/t
