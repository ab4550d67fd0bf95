export TMPDIR=/tmp
mkdir -p gpurun_out/r05z
source tools/gpu_step.sh
step 600 gpurun_out/r05z/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sine_elu.py tests/test_gpu_parity.py -k "sine_elu or critic_grad or actor_grad"
tail -3 gpurun_out/r05z/tests.log
for i in 1 2; do
  step 300 gpurun_out/r05z/bench_$i.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 128,4096 --extra-systems car_park
  python3 tools/bench_summary.py gpurun_out/r05z/bench_$i.log
done
