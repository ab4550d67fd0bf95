export TMPDIR=/tmp
mkdir -p gpurun_out/r05r
source tools/gpu_step.sh
step 1000 gpurun_out/r05r/tests.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu
tail -3 gpurun_out/r05r/tests.log
i=0
for e in "CACTO_PIPE_DEVWAIT=3" "CACTO_PIPE_DEVWAIT=1" "CACTO_PIPE_DEVWAIT=3" "CACTO_PIPE_DEVWAIT=1"; do
  i=$((i+1))
  step 300 gpurun_out/r05r/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 128,4096 --extra-systems manipulator,car_park,ur5
  echo "== $i $e" >> gpurun_out/r05r/summary.txt; python3 tools/bench_summary.py gpurun_out/r05r/bench_${i}.log >> gpurun_out/r05r/summary.txt || true
done
cat gpurun_out/r05r/summary.txt
echo done
