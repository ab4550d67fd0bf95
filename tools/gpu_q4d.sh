# q4 quick iteration: chain phase stamps, update rates (no tests)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/q4d
mkdir -p $D
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py > $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor double_integrator >> $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor manipulator >> $D/stamps.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,ur5 --batches 128 > $D/bench.json 2> $D/bench.err
