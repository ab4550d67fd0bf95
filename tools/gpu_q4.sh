# q4 (4-sample tile) learner chains: update parity / pipeline tests, then the update rates with the
# q4 chains (default), with the 16-sample chains everywhere, and with q4 at every batch size.
# Test failures (pytest rc 1) do not stop the benches; anything else (timeout, fault) does.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_nan_abort.py tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_main_loop.py tests/test_gpu_dp.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/q4_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,car_park > gpurun_out/q4_bench.json 2> gpurun_out/q4_bench.err &&
CACTO_Q4_MAX_BP=0 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,car_park > gpurun_out/q16_bench.json 2> gpurun_out/q16_bench.err &&
CACTO_Q4_MAX_BP=100000 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-diagnostics --no-config0 --extra-systems manipulator,car_park > gpurun_out/q4all_bench.json 2> gpurun_out/q4all_bench.err
