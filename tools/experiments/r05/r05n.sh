export TMPDIR=/tmp
mkdir -p gpurun_out/r05n
source tools/gpu_step.sh
step 900 gpurun_out/r05n/tests.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "per_" tests/test_gpu_per_pipeline.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py
tail -2 gpurun_out/r05n/tests.log
step 120 gpurun_out/r05n/stamps_8192.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python tools/per_stamps.py
step 120 gpurun_out/r05n/stamps_4096.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so CACTO_PER_TOP=4096 python tools/per_stamps.py
grep -h "per workgroup" gpurun_out/r05n/stamps_*.log
for i in 1 2; do
  step 300 gpurun_out/r05n/bench_${i}.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i" >> gpurun_out/r05n/summary.txt; python3 tools/bench_summary.py gpurun_out/r05n/bench_${i}.log >> gpurun_out/r05n/summary.txt || true
done
cat gpurun_out/r05n/summary.txt
echo done
