export TMPDIR=/tmp
mkdir -p gpurun_out/r05y
source tools/gpu_step.sh
for e in "CACTO_HIP_LIB=cacto_amd/libcacto_noelu.so" "CACTO_X=1" "CACTO_HIP_LIB=cacto_amd/libcacto_noelu.so" "CACTO_X=1"; do
  step 300 gpurun_out/r05y/bench.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems=
  echo "== $e"; python3 tools/bench_summary.py gpurun_out/r05y/bench.log | grep "B=4096"
done
