# per-system rollout choices: parity tests + rollout rates of every system
set -e
mkdir -p gpurun_out/r3d
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nan_abort.py tests/test_gpu_rl_solve.py tests/test_gpu_fullsize.py tests/test_gpu_env_surface.py > gpurun_out/r3d/tests.log 2>&1
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --update-steps 20 --batches "" --long-steps 300 > gpurun_out/r3d/$v.json 2> gpurun_out/r3d/$v.err
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/r3d/$v.json').read().strip().splitlines()[-1])
print('$v', 'DI %.1f M (kern %.4f ms, long %.1f M)' % (d['value']/1e6, d['roofline']['kernel_ms'], d['long_region']['median']/1e6),
      ' '.join('%s %.1f M (%.4f ms)' % (s, e['long_region']['median']/1e6, e['rollout_kernel_ms']) for s, e in d['extra_systems'].items()))
" >> gpurun_out/r3d/summary.txt
done
