export TMPDIR=/tmp
mkdir -p gpurun_out/r05u
source tools/gpu_step.sh
step 900 gpurun_out/r05u/tests.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_per_pipeline.py tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py
tail -2 gpurun_out/r05u/tests.log
step 900 gpurun_out/r05u/pmc.log bash tools/r05t.sh
tail -12 gpurun_out/r05u/pmc.log
