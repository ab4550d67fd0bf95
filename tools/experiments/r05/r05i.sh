export TMPDIR=/tmp
mkdir -p gpurun_out/r05i
source tools/gpu_step.sh
step 600 gpurun_out/r05i/tests.log python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_parity.py -k "per_" tests/test_gpu_per_pipeline.py tests/test_gpu_fullsize.py tests/test_gpu_relo.py
tail -3 gpurun_out/r05i/tests.log
for e in "CACTO_PER_DEEP_TOP=1" "CACTO_PER_DEEP_TOP=0" "CACTO_PER_FUSED=0"; do
  step 120 gpurun_out/r05i/micro_$e.log env $e python tools/per_micro.py 4096 300
  echo "== $e" >> gpurun_out/r05i/micro.txt; cat gpurun_out/r05i/micro_$e.log | grep "us per call" >> gpurun_out/r05i/micro.txt
done
cat gpurun_out/r05i/micro.txt
i=0
for e in "CACTO_PER_DEEP_TOP=1" "CACTO_PER_DEEP_TOP=0" "CACTO_PER_DEEP_TOP=1" "CACTO_PER_DEEP_TOP=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05i/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05i/summary.txt; python3 tools/bench_summary.py gpurun_out/r05i/bench_${i}.log >> gpurun_out/r05i/summary.txt || true
done
cat gpurun_out/r05i/summary.txt
step 300 gpurun_out/r05i/prof_cp.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05i/pcp -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems car_park --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05i/pcp/run_results.db > gpurun_out/r05i/cp_stats.csv
python3 tools/timeline.py gpurun_out/r05i/pcp/run_results.db k_ 40 300 > gpurun_out/r05i/cp_timeline_per.txt
rm -rf gpurun_out/r05i/pcp
cat gpurun_out/r05i/cp_timeline_per.txt
echo done
