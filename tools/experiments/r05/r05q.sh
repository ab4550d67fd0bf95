export TMPDIR=/tmp
mkdir -p gpurun_out/r05q
source tools/gpu_step.sh
step 900 gpurun_out/r05q/tests.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_parity.py -k "per_ or pipelined"
tail -2 gpurun_out/r05q/tests.log
i=0
for e in "CACTO_PIPE_DEVWAIT=3" "CACTO_PIPE_DEVWAIT=1" "CACTO_PIPE_DEVWAIT=3" "CACTO_PIPE_DEVWAIT=1"; do
  i=$((i+1))
  step 300 gpurun_out/r05q/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05q/summary.txt; python3 tools/bench_summary.py gpurun_out/r05q/bench_${i}.log >> gpurun_out/r05q/summary.txt || true
done
cat gpurun_out/r05q/summary.txt
step 300 gpurun_out/r05q/prof_di.log env CACTO_PIPE_DEVWAIT=3 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q/pdi -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/timeline.py gpurun_out/r05q/pdi/run_results.db k_ 30 200 > gpurun_out/r05q/di_timeline.txt
rm -rf gpurun_out/r05q/pdi
cat gpurun_out/r05q/di_timeline.txt
echo done
