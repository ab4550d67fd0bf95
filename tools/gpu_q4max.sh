# 4-sample-tile chains above B = 512: DI B = 1024 / 2048 and UR5 B = 2048 with CACTO_Q4_MAX_BP 512 (default) / 2048
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/q4max
mkdir -p $D
for m in 512 2048; do
  CACTO_Q4_MAX_BP=$m timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 1024,2048 --update-steps 500 --extra-systems ur5 > $D/b$m.json 2> $D/b$m.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$m.json').read().strip().splitlines()[-1])
print('q4max $m', {k: round(v['value']) for k, v in d['critic_updates'].items()}, {s: {k: round(v['value']) for k, v in e['critic_updates'].items()} for s, e in d['extra_systems'].items()})
" >> $D/summary.txt
done
