# phase stamps (CACTO_STAMPS diagnostic build): critic chain, actor chains, rollout step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so
timeout -k 10 120 python -u tools/critic_stamps.py > gpurun_out/stamps.log 2>&1 &&
timeout -k 10 120 python -u tools/critic_stamps.py actor double_integrator >> gpurun_out/stamps.log 2>&1 &&
timeout -k 10 120 python -u tools/critic_stamps.py actor manipulator >> gpurun_out/stamps.log 2>&1 &&
timeout -k 10 120 python -u tools/rollout_stamps.py double_integrator >> gpurun_out/stamps.log 2>&1 &&
timeout -k 10 120 python -u tools/rollout_stamps.py ur5 2048 >> gpurun_out/stamps.log 2>&1
