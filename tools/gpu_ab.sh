# Rollout A/B of library variants side by side: the bench's rollout rates of every system, each
# variant run twice in alternation. Usage: bash tools/gpu_ab.sh cacto_amd/libA.so cacto_amd/libB.so ...
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for L in "$@"; do
    v=$(basename $L .so)_$rep
    CACTO_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --update-steps 20 --batches "" --long-steps 300 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/$v.json').read().strip().splitlines()[-1])
print('$v', 'DI %.1f M (kern %.4f ms, long %.1f M)' % (d['value']/1e6, d['roofline']['kernel_ms'], d['long_region']['median']/1e6),
      ' '.join('%s %.1f M (%.4f ms)' % (s, e['long_region']['median']/1e6, e['rollout_kernel_ms']) for s, e in d['extra_systems'].items()))
" >> gpurun_out/ab/summary.txt
  done
done
