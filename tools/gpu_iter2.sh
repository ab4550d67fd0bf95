# learner tests, critic/actor stamps, the full bench (long region included)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_upd.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/critic_stamps.py > gpurun_out/stamps.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 > gpurun_out/bench_it.json 2> gpurun_out/bench_it.err
