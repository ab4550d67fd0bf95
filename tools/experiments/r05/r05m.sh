export TMPDIR=/tmp
mkdir -p gpurun_out/r05m
source tools/gpu_step.sh
step 120 gpurun_out/r05m/stamps_8192.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python tools/per_stamps.py
step 120 gpurun_out/r05m/stamps_4096.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so CACTO_PER_TOP=4096 python tools/per_stamps.py
cat gpurun_out/r05m/stamps_*.log | grep -v amdgpu.ids
step 300 gpurun_out/r05m/prof_mn.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05m/pmn -o run -- python3 bench.py --system manipulator --rollouts 8192 --steps 2 --warmup 1 --update-steps 200 --batches 8192 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05m/pmn/run_results.db > gpurun_out/r05m/mn_stats.csv
python3 tools/timeline.py gpurun_out/r05m/pmn/run_results.db k_ 40 200 > gpurun_out/r05m/mn_timeline.txt
rm -rf gpurun_out/r05m/pmn
step 300 gpurun_out/r05m/prof_di.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05m/pdi -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 200 --batches 4096 --extra-systems= --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0
python3 tools/prof_summary.py stats gpurun_out/r05m/pdi/run_results.db > gpurun_out/r05m/di_stats.csv
python3 tools/timeline.py gpurun_out/r05m/pdi/run_results.db k_ 40 200 > gpurun_out/r05m/di_timeline.txt
rm -rf gpurun_out/r05m/pdi
echo done
