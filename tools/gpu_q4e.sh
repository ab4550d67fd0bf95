# q4 L2 warm-up: update rates with and without the prefetch workgroups, chain stamps (pair)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/q4e
mkdir -p $D
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,ur5 --batches 128 > $D/bench.json 2> $D/bench.err &&
CACTO_Q4_PREFETCH=0 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator --batches 128 > $D/bench_nopf.json 2> $D/bench_nopf.err &&
CACTO_Q4_PREFETCH=24 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator --batches 128 > $D/bench_pf24.json 2> $D/bench_pf24.err &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py pair > $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor manipulator >> $D/stamps.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_main_loop.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $D/tests.log 2>&1
