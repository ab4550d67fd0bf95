# Rollout schedules: rollout parity tests, k_rollout time per schedule (tools/ro_sched.py), k_rollout_ks phase stamps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ws
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nan_abort.py tests/test_gpu_dp.py tests/test_gpu_relo.py -k "rollout or status or kept or ep0 or rccl or relo" > gpurun_out/ws/tests.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py double_integrator 4096 "0,0 -1,0 -3,0 2,0" > gpurun_out/ws/sched.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py car_park 4096 "0,0 -1,0 -3,0" >> gpurun_out/ws/sched.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py single_integrator 4096 "0,0 -1,0 -3,0" >> gpurun_out/ws/sched.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py car 4096 "0,0 -1,0 -3,0" >> gpurun_out/ws/sched.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/tt_stamps.py double_integrator ks > gpurun_out/ws/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py ur5 2048 >> gpurun_out/ws/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py manipulator 8192 >> gpurun_out/ws/stamps.log 2>&1
