export TMPDIR=/tmp
mkdir -p gpurun_out/r05l
source tools/gpu_step.sh
i=0
for e in "CACTO_PER_OVERLAP=1" "CACTO_PER_OVERLAP=0" "CACTO_PER_OVERLAP=1" "CACTO_PER_OVERLAP=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05l/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05l/summary.txt; python3 tools/bench_summary.py gpurun_out/r05l/bench_${i}.log >> gpurun_out/r05l/summary.txt || true
done
cat gpurun_out/r05l/summary.txt
step 300 gpurun_out/r05l/prof_cp.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05l/pcp -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems car_park --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05l/pcp/run_results.db > gpurun_out/r05l/cp_stats.csv
python3 tools/timeline.py gpurun_out/r05l/pcp/run_results.db k_ 40 300 > gpurun_out/r05l/cp_timeline_per.txt
rm -rf gpurun_out/r05l/pcp
cat gpurun_out/r05l/cp_timeline_per.txt
echo done
