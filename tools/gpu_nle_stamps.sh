# UR5 rollout step stamps, RNEA split vs serial
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/nle
mkdir -p $D
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 200 python -u tools/rollout_stamps.py ur5 2048 > $D/stamps_split.txt 2>&1 || exit 1
CACTO_RO_NLE_SERIAL=1 CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 200 python -u tools/rollout_stamps.py ur5 2048 > $D/stamps_serial.txt 2>&1
