# B=4096 updates: side-stream priority variants, then one kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pr
for pr in none hi lo; do
  CACTO_SIDE_PRIO=$pr timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 4096 --update-steps 500 --extra-systems manipulator > gpurun_out/pr/b$pr.json 2> gpurun_out/pr/b$pr.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/pr/b$pr.json').read().strip().splitlines()[-1])
m=d['extra_systems']['manipulator']['critic_updates']
print('prio $pr', 'DI B=4096 %.0f' % d['critic_updates']['B=4096']['value'], 'manip', {k: round(v['value']) for k, v in m.items()})
" >> gpurun_out/pr/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pr/prof -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 4096 --update-steps 500 --extra-systems "" > gpurun_out/pr/prof.log 2>&1
