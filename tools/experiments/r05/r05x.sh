export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
source tools/gpu_step.sh
echo "AMD_SERIALIZE_KERNEL=${AMD_SERIALIZE_KERNEL-unset} HIP_LAUNCH_BLOCKING=${HIP_LAUNCH_BLOCKING-unset} CACTO_PIPE_DEVWAIT=${CACTO_PIPE_DEVWAIT-unset}"
for e in "CACTO_X=0" "CACTO_PIPE_DEVWAIT=3" "CACTO_PIPE_DEVWAIT=1"; do
  step 300 gpurun_out/r05x/bench_$e.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems=
  echo "== $e"; python3 tools/bench_summary.py gpurun_out/r05x/bench_$e.log
done
