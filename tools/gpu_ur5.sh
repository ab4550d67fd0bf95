set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ur5 or rollout or manipulator" > gpurun_out/gpu_ur5.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py ur5 2048 > gpurun_out/ro_stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py manipulator 4096 >> gpurun_out/ro_stamps.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config0 > gpurun_out/bench_ur5.json 2> gpurun_out/bench_ur5.err
