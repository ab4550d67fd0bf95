# learner at large batches: update tests, then B=4096 / 8192 update rates per wgrad chunk size
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/as
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/as/tests.log 2>&1 || exit 1
for ch in 0 256 512; do
  CACTO_WG_CHUNK=$ch timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 4096 --update-steps 500 --extra-systems manipulator > gpurun_out/as/b$ch.json 2> gpurun_out/as/b$ch.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/as/b$ch.json').read().strip().splitlines()[-1])
m=d['extra_systems']['manipulator']['critic_updates']
print('chunk $ch', 'DI B=4096 %.0f' % d['critic_updates']['B=4096']['value'], 'manip', {k: round(v['value']) for k, v in m.items()})
" >> gpurun_out/as/summary.txt
done
