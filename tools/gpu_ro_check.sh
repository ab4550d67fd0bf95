# rollout parity tests, phase stamps of the rollout step, and the rollout rates of the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rollout or plot or create_TO" --timeout 200 --timeout-method thread > gpurun_out/gpu_ro.log 2>&1 &&
for s in double_integrator manipulator ur5; do CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py $s >> gpurun_out/stamps_new.log 2>&1 || exit 1; done &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-diagnostics --batches 128 --update-steps 20 > gpurun_out/bench_ro.json 2> gpurun_out/bench_ro.err
