export TMPDIR=/tmp
mkdir -p gpurun_out/r05h
source tools/gpu_step.sh
step 600 gpurun_out/r05h/tests.log python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_update_parity.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py
tail -3 gpurun_out/r05h/tests.log
i=0
for e in "CACTO_WGB_AHEAD=6" "CACTO_WGB_AHEAD=3" "CACTO_WG_CHUNK=512" "CACTO_WGB_AHEAD=6" "CACTO_WGB_AHEAD=3" "CACTO_WG_CHUNK=512"; do
  i=$((i+1))
  step 300 gpurun_out/r05h/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator,car_park
  echo "== $i $e" >> gpurun_out/r05h/summary.txt; python3 tools/bench_summary.py gpurun_out/r05h/bench_${i}.log >> gpurun_out/r05h/summary.txt || true
done
cat gpurun_out/r05h/summary.txt
step 300 gpurun_out/r05h/prof_cp.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05h/pcp -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems car_park --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05h/pcp/run_results.db > gpurun_out/r05h/cp_stats.csv
python3 tools/timeline.py gpurun_out/r05h/pcp/run_results.db k_ 70 300 > gpurun_out/r05h/cp_timeline_per.txt
rm -rf gpurun_out/r05h/pcp
head -30 gpurun_out/r05h/cp_stats.csv
echo done
