export TMPDIR=/tmp
mkdir -p gpurun_out/r05k
source tools/gpu_step.sh
step 900 gpurun_out/r05k/tests.log python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_relo.py tests/test_gpu_main_loop.py
tail -3 gpurun_out/r05k/tests.log
grep -q " passed" gpurun_out/r05k/tests.log || exit 3
grep -q "failed" gpurun_out/r05k/tests.log && exit 4
i=0
for e in "CACTO_PER_OVERLAP=1" "CACTO_PER_OVERLAP=0" "CACTO_PER_OVERLAP=1" "CACTO_PER_OVERLAP=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05k/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05k/summary.txt; python3 tools/bench_summary.py gpurun_out/r05k/bench_${i}.log >> gpurun_out/r05k/summary.txt || true
done
cat gpurun_out/r05k/summary.txt
step 300 gpurun_out/r05k/prof_cp.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05k/pcp -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems car_park --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05k/pcp/run_results.db > gpurun_out/r05k/cp_stats.csv
python3 tools/timeline.py gpurun_out/r05k/pcp/run_results.db k_ 40 300 > gpurun_out/r05k/cp_timeline_per.txt
rm -rf gpurun_out/r05k/pcp
cat gpurun_out/r05k/cp_timeline_per.txt
echo done
