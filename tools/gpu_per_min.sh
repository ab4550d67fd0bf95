# car_park PER update rates with the multi-workgroup PER kernels from B = 1 / 64 / 512 (default)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/permin
mkdir -p $D
for m in 1 128 512; do
  CACTO_PER_MW_MIN=$m timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 1000 --extra-systems car_park > $D/b$m.json 2> $D/b$m.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$m.json').read().strip().splitlines()[-1])
print('mw_min $m', {s: {k: round(v['value']) for k, v in e['critic_updates'].items()} for s, e in d['extra_systems'].items()})
" >> $D/summary.txt
done
