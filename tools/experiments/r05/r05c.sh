export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
source tools/gpu_step.sh
step 300 gpurun_out/r05c/tests_sw.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "slot_refill or rewards_separate or per_step"
tail -3 gpurun_out/r05c/tests_sw.log
step 300 gpurun_out/r05c/tests_fs.log python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py -k "rollout or fullsize_update"
tail -3 gpurun_out/r05c/tests_fs.log
step 200 gpurun_out/r05c/stamps_sw.log env CACTO_HIP_LIB=cacto_amd/libcacto_diag.so python -u tools/sw_stamps.py manipulator 8192
cat gpurun_out/r05c/stamps_sw.log
i=0
for e in "CACTO_RO_SW=1" "CACTO_RO_SW=0" "CACTO_WG_PERM=0" "CACTO_WG_CHUNK=128" "CACTO_WG_CHUNK=512" "CACTO_RO_SW=1" "CACTO_RO_SW=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05c/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator
  echo "== $i $e" >> gpurun_out/r05c/summary.txt; python3 tools/bench_summary.py gpurun_out/r05c/bench_${i}.log >> gpurun_out/r05c/summary.txt || true
done
cat gpurun_out/r05c/summary.txt
for e in "CACTO_PER_PRIO=1" "CACTO_PER_PRIO=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05c/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems car_park
  echo "== $i $e" >> gpurun_out/r05c/summary.txt; python3 tools/bench_summary.py gpurun_out/r05c/bench_${i}.log >> gpurun_out/r05c/summary.txt || true
done
cat gpurun_out/r05c/summary.txt
