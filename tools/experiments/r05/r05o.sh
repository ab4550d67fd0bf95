export TMPDIR=/tmp
mkdir -p gpurun_out/r05o
source tools/gpu_step.sh
step 120 gpurun_out/r05o/stamps_8192.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python tools/per_stamps.py
step 120 gpurun_out/r05o/stamps_4096.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so CACTO_PER_TOP=4096 python tools/per_stamps.py
grep -h "per workgroup\|thread 0" gpurun_out/r05o/stamps_*.log
