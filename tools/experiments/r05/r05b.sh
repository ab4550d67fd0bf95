export TMPDIR=/tmp
mkdir -p gpurun_out/r05b
source tools/gpu_step.sh
step 300 gpurun_out/r05b/tests_sw.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "slot_refill or rewards_separate"
tail -3 gpurun_out/r05b/tests_sw.log
step 800 gpurun_out/r05b/tests.log python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_per_pipeline.py tests/test_gpu_graph.py tests/test_gpu_relo.py tests/test_gpu_dp.py
tail -3 gpurun_out/r05b/tests.log
i=0
for e in "CACTO_WG_BIG=1" "CACTO_WG_BIG=0" "CACTO_PIPE_DEVWAIT=1" "CACTO_RO_SW=1"; do
  i=$((i+1))
  step 300 gpurun_out/r05b/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park,manipulator
  echo "== $i $e" >> gpurun_out/r05b/summary.txt; python3 tools/bench_summary.py gpurun_out/r05b/bench_${i}.log >> gpurun_out/r05b/summary.txt || true
done
cat gpurun_out/r05b/summary.txt
step 200 gpurun_out/r05b/stamps_sw.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python -u tools/sw_stamps.py manipulator 8192
cat gpurun_out/r05b/stamps_sw.log
step 300 gpurun_out/r05b/prof_seq.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05b/pseq -o run -- python3 bench.py --steps 3 --warmup 1 --update-steps 200 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 --graph
python3 tools/prof_summary.py stats gpurun_out/r05b/pseq/run_results.db > gpurun_out/r05b/pseq_stats.csv
python3 tools/timeline.py gpurun_out/r05b/pseq/run_results.db k_ 40 30 > gpurun_out/r05b/pseq_timeline.txt
rm -rf gpurun_out/r05b/pseq
step 300 gpurun_out/r05b/prof_pipe.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05b/ppipe -o run -- python3 bench.py --steps 3 --warmup 1 --update-steps 200 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05b/ppipe/run_results.db > gpurun_out/r05b/ppipe_stats.csv
python3 tools/timeline.py gpurun_out/r05b/ppipe/run_results.db k_ 40 40 > gpurun_out/r05b/ppipe_timeline.txt
rm -rf gpurun_out/r05b/ppipe
head -8 gpurun_out/r05b/pseq_stats.csv
