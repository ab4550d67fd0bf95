# rollout iteration: parity / full-size tests, step stamps, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_main_loop.py tests/test_gpu_rl_solve.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_ro.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py double_integrator > gpurun_out/ro_stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py car_park >> gpurun_out/ro_stamps.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline --no-config0 --update-steps 100 > gpurun_out/bench_ro.json 2> gpurun_out/bench_ro.err
