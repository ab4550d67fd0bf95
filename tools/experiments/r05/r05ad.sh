# the side stream's wait as a kernel (CACTO_PIPE_WAITK): pipeline identity tests, then manipulator A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ad
source tools/gpu_step.sh
step 600 gpurun_out/r05ad/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_update_parity.py tests/test_gpu_fullsize.py
tail -3 gpurun_out/r05ad/tests.log
grep -q " passed" gpurun_out/r05ad/tests.log && ! grep -q " failed" gpurun_out/r05ad/tests.log || exit 1
for rep in 1 2; do
  for E in "X=0" "CACTO_PIPE_WAITK=0"; do
    v=$(echo "$E" | tr '= ' '__')_$rep
    export $E
    step 300 gpurun_out/r05ad/$v.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator
    unset ${E%%=*}
    echo "$v $(python3 tools/bench_summary.py gpurun_out/r05ad/$v.log | tr '\n' ' ')" >> gpurun_out/r05ad/summary.txt
  done
done
cat gpurun_out/r05ad/summary.txt
