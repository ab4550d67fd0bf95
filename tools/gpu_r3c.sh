# rollout slot registers + strip GEMM check: parity, NaN, update parity, full-size; stamps; bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nan_abort.py tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_graph.py > gpurun_out/r3c/tests.log 2>&1
for s in double_integrator manipulator ur5; do
  CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python tools/rollout_stamps.py $s >> gpurun_out/r3c/stamps.log 2>&1
done
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --update-steps 300 > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err
