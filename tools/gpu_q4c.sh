# q4 iteration: learner parity, update rates (PER two-stream vs paired), chain phase stamps
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/q4c
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_main_loop.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $D/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,car_park,ur5 --batches 128 > $D/bench.json 2> $D/bench.err &&
CACTO_PER_PAIRED=1 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems car_park --batches 128 > $D/bench_perpair.json 2> $D/bench_perpair.err &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py > $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor double_integrator >> $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor manipulator >> $D/stamps.log 2>&1
