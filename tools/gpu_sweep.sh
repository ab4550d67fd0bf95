set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_chain_iter.sh &&
timeout -k 10 120 python -u tools/ro_sched.py ur5 2048 "0,0 1,256 1,512 2,256 2,128 4,128 4,64" > gpurun_out/sched.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py double_integrator 4096 "0,0 1,256 2,256 4,256 4,128" >> gpurun_out/sched.log 2>&1 &&
timeout -k 10 120 python -u tools/ro_sched.py manipulator 8192 "0,0 1,256 2,256 4,256 4,128" >> gpurun_out/sched.log 2>&1
