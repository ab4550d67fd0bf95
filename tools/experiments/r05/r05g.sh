export TMPDIR=/tmp
mkdir -p gpurun_out/r05g
source tools/gpu_step.sh
step 600 gpurun_out/r05g/tests.log python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_parity.py -k "per_" tests/test_gpu_fullsize.py tests/test_gpu_per_pipeline.py tests/test_gpu_dp.py
tail -3 gpurun_out/r05g/tests.log
i=0
for e in "CACTO_PER_DEEP_TOP=1" "CACTO_PER_DEEP_TOP=0" "CACTO_PER_DEEP_TOP=1" "CACTO_PER_DEEP_TOP=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05g/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05g/summary.txt; python3 tools/bench_summary.py gpurun_out/r05g/bench_${i}.log >> gpurun_out/r05g/summary.txt || true
done
cat gpurun_out/r05g/summary.txt
step 300 gpurun_out/r05g/prof_cp.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05g/pcp -o run -- python3 bench.py --system car_park --steps 3 --warmup 1 --update-steps 200 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05g/pcp/run_results.db > gpurun_out/r05g/cp_stats.csv
python3 tools/timeline.py gpurun_out/r05g/pcp/run_results.db k_ 60 40 > gpurun_out/r05g/cp_timeline.txt
rm -rf gpurun_out/r05g/pcp
head -20 gpurun_out/r05g/cp_stats.csv
echo done
