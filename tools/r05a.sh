export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
source tools/gpu_step.sh
step 600 gpurun_out/r05a/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_relo.py tests/test_gpu_per_pipeline.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py
i=0
for f in 1 0 1 0; do
  i=$((i+1))
  step 300 gpurun_out/r05a/bench_${i}_f$f.log env CACTO_PER_FUSED=$f python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
done
tail -3 gpurun_out/r05a/tests.log
