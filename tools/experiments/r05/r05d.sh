export TMPDIR=/tmp
mkdir -p gpurun_out/r05d
source tools/gpu_step.sh
step 400 gpurun_out/r05d/tests.log python -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_gpu_per_pipeline.py
tail -3 gpurun_out/r05d/tests.log
i=0
for e in "CACTO_PIPE_SIGNAL=0" "CACTO_PIPE_SIGNAL=1" "CACTO_WG_CHUNK=256" "CACTO_PIPE_SIGNAL=0" "CACTO_PIPE_SIGNAL=1" "CACTO_WG_CHUNK=256"; do
  i=$((i+1))
  step 300 gpurun_out/r05d/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator,car_park
  echo "== $i $e" >> gpurun_out/r05d/summary.txt; python3 tools/bench_summary.py gpurun_out/r05d/bench_${i}.log >> gpurun_out/r05d/summary.txt || true
done
cat gpurun_out/r05d/summary.txt
