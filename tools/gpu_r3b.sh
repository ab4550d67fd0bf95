# round-3: rewards kernel check + bench + the round profile set
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nan_abort.py > gpurun_out/r3b/tests.log 2>&1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config0 --update-steps 300 --extra-systems ur5 > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err
bash tools/prof_round.sh r03 > gpurun_out/r3b/prof.log 2>&1
