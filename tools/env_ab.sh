# Learner A/B of environment settings on one library: the bench's update rates per setting, each
# run twice in alternation. Usage: bash tools/env_ab.sh "VAR=a" "VAR=b" ...
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/eab
for rep in 1 2; do
  for E in "$@"; do
    v=$(echo "$E" | tr '= ' '__')_$rep
    env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 > gpurun_out/eab/$v.json 2> gpurun_out/eab/$v.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/eab/$v.json').read().strip().splitlines()[-1])
print('$v', ' '.join('%s %.0f' % (k.replace('_updates_per_s', ''), v) for k, v in d.items() if 'updates_per_s' in k))
" >> gpurun_out/eab/summary.txt
  done
done
