# round-end set, then UR5 rollout stamps (RNEA vs CRBA split). Usage: bash tools/gpu_round_end_ur5.sh r02
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python -u tools/rollout_stamps.py ur5 2048 > gpurun_out/ro_stamps.log 2>&1 &&
bash tools/gpu_round_end.sh ${1:-r02}
