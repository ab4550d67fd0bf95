# Learner A/B of library variants: the bench's update rates (DI B = 128 / 4096 and every extra
# system at its configs' batches), each variant run twice in alternation.
# Usage: bash tools/upd_ab.sh cacto_amd/libA.so cacto_amd/libB.so ...
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/uab
for rep in 1 2; do
  for L in "$@"; do
    v=$(basename $L .so)_$rep
    CACTO_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --update-steps 400 > gpurun_out/uab/$v.json 2> gpurun_out/uab/$v.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/uab/$v.json').read().strip().splitlines()[-1])
print('$v', ' '.join('%s %.0f' % (k.replace('_updates_per_s', ''), v) for k, v in d.items() if 'updates_per_s' in k))
" >> gpurun_out/uab/summary.txt
  done
done
