# the round's new GPU test files first (the env-surface file, newest kernel code, in its own run
# last), then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_update_parity.py tests/test_gpu_main_loop.py tests/test_gpu_graph.py tests/test_gpu_dp.py -v --timeout 240 --timeout-method thread > gpurun_out/gpu_new.log 2>&1
rc=$?
echo "first rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_env_surface.py -v --timeout 120 --timeout-method thread > gpurun_out/gpu_env.log 2>&1
  rc2=$?
  echo "env rc=$rc2"
  if [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
    echo "all rc=$?"
  fi
fi
