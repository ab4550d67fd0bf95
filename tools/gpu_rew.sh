# compacted rewards pass + layer 3 on wave 0 of each rollout team: rollout parity tests, then
# rollout rates for: new/new, team layer 3 + compacted rewards, team layer 3 + [b][t] rewards
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/rew
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nan_abort.py tests/test_gpu_rl_solve.py tests/test_gpu_fullsize.py tests/test_gpu_env_surface.py tests/test_gpu_main_loop.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
for v in new l3team old; do
  unset CACTO_REW_GRID_BT CACTO_RO_L3_TEAM
  if [ $v = l3team ]; then export CACTO_RO_L3_TEAM=1; fi
  if [ $v = old ]; then export CACTO_RO_L3_TEAM=1 CACTO_REW_GRID_BT=1; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 300 --batches "" --update-steps 20 > $D/b$v.json 2> $D/b$v.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$v.json').read().strip().splitlines()[-1])
r=d['roofline']
print('$v DI %.1f M (long %.1f M) k_rollout %.4f ms rewards %.4f ms batch %.4f ms' % (d['value']/1e6, d['long_region']['median']/1e6, r['kernel_ms'], r['rewards_kernel_ms'], r['rollout_batch_ms']),
      ' '.join('%s %.1f M' % (s, e['long_region']['median']/1e6) for s, e in d['extra_systems'].items()))
" >> $D/summary.txt
done
