# placement prefetch in the chain RNEA / CRBA: rollout parity tests, UR5 / manipulator rates
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/pf
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nan_abort.py tests/test_gpu_fullsize.py tests/test_gpu_env_surface.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 100 --batches "" --update-steps 20 --extra-systems ur5,manipulator > $D/b.json 2> $D/b.err || exit 1
python3 -c "
import json
d=json.loads(open('$D/b.json').read().strip().splitlines()[-1])
print('pf', ' '.join('%s %.1f M (%.4f ms)' % (s, e['long_region']['median']/1e6, e['rollout_kernel_ms']) for s, e in d['extra_systems'].items()))
" >> $D/summary.txt
