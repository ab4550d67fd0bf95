export TMPDIR=/tmp
mkdir -p gpurun_out/r05f
source tools/gpu_step.sh
step 600 gpurun_out/r05f/tests.log python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_graph.py
tail -3 gpurun_out/r05f/tests.log
i=0
for e in "CACTO_CHAIN_XCD=1" "CACTO_CHAIN_XCD=0" "CACTO_CHAIN_XCD=1" "CACTO_CHAIN_XCD=0"; do
  i=$((i+1))
  step 300 gpurun_out/r05f/bench_${i}.log env $e python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 --batches 4096 --extra-systems manipulator,car_park
  echo "== $i $e" >> gpurun_out/r05f/summary.txt; python3 tools/bench_summary.py gpurun_out/r05f/bench_${i}.log >> gpurun_out/r05f/summary.txt || true
done
cat gpurun_out/r05f/summary.txt
A="--steps 3 --warmup 1 --extra-systems= --update-steps 20 --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 --batches 4096"
for x in 1 0; do
  step 120 gpurun_out/r05f/pmc_fetch_x$x.log env CACTO_CHAIN_XCD=$x rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_wgrad|k_adam|k_critic|k_actor" -d gpurun_out/r05f/pf$x -o run -- python3 bench.py $A
  python3 tools/prof_summary.py pmc gpurun_out/r05f/pf$x/run_results.db > gpurun_out/r05f/pmc_learn_fetch_b4096_x$x.csv
  rm -rf gpurun_out/r05f/pf$x
done
cat gpurun_out/r05f/pmc_learn_fetch_b4096_x*.csv
step 600 gpurun_out/r05f/bench_gpus2.log env CACTO_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 100 --extra-systems car_park
grep -o '"loop": "[a-z_]*"' gpurun_out/r05f/bench_gpus2.log | sort | uniq -c
