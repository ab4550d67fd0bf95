# manipulator B = 8192 learner: side-stream priority and stream-value signalling A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ab
source tools/gpu_step.sh
for rep in 1 2; do
  for E in "X=0" "CACTO_SIDE_PRIO=lo" "CACTO_SIDE_PRIO=hi" "CACTO_PIPE_SIGNAL=1"; do
    v=$(echo "$E" | tr '= ' '__')_$rep
    export $E
    step 300 gpurun_out/r05ab/$v.log python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator
    unset ${E%%=*}
    echo "$v $(python3 tools/bench_summary.py gpurun_out/r05ab/$v.log | tr '\n' ' ')" >> gpurun_out/r05ab/summary.txt
  done
done
cat gpurun_out/r05ab/summary.txt
