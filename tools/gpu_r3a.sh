# round-3 check: DP / main loop / NaN / rollout parity tests, rollout stamps, a short bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_main_loop.py tests/test_gpu_nan_abort.py tests/test_gpu_parity.py > gpurun_out/r3a/tests.log 2>&1
for s in double_integrator manipulator car_park ur5; do
  CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python tools/rollout_stamps.py $s >> gpurun_out/r3a/stamps.log 2>&1
done
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config0 --update-steps 300 > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err
