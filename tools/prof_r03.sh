# r03 learner profile at the reference batch: kernel trace (DI B = 128, manipulator B = 64 via the
# bench's extra systems), the gaps between the update kernels, and per-phase stamps of the q4 chains
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/prof_r03
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t128 -o run -- python3 bench.py --steps 5 --warmup 2 --update-steps 1000 --batches 128 --extra-systems manipulator --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 > $D/b128.json 2> $D/b128.err &&
python3 tools/prof_summary.py stats $D/t128/run_results.db > $D/stats_b128.csv &&
python3 tools/prof_gaps.py $D/t128/run_results.db > $D/gaps_b128.txt &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py > $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor double_integrator >> $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py actor manipulator >> $D/stamps.log 2>&1 &&
CACTO_HIP_LIB=cacto_amd/libcacto_hip_stamps.so timeout -k 10 120 python3 -u tools/critic_stamps.py pair >> $D/stamps.log 2>&1
