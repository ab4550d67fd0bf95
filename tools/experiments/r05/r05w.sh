export TMPDIR=/tmp
mkdir -p gpurun_out/r05w
source tools/gpu_step.sh
step 600 gpurun_out/r05w/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sine_elu or critic_grad or actor_grad or forward_and_input or update_matches"
tail -3 gpurun_out/r05w/tests.log
for i in 1 2; do
  step 300 gpurun_out/r05w/bench_$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --extra-systems car_park
  python3 tools/bench_summary.py gpurun_out/r05w/bench_$i.log
done
