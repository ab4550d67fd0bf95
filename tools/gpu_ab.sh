# rollout A/B: the library variants side by side (rollout rates of every system)
set -e
mkdir -p gpurun_out/ab
for v in main np nr nn main; do
  if [ $v = main ]; then L=cacto_amd/libcacto_hip.so; else L=cacto_amd/libro_$v.so; fi
  CACTO_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --update-steps 20 --batches "" --long-steps 300 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab/$v.json').read().strip().splitlines()[-1])
print('$v', 'DI %.1f M (kern %.4f ms, long %.1f M)' % (d['value']/1e6, d['roofline']['kernel_ms'], d['long_region']['median']/1e6),
      ' '.join('%s %.1f M (%.4f ms)' % (s, e['long_region']['median']/1e6, e['rollout_kernel_ms']) for s, e in d['extra_systems'].items()))
" >> gpurun_out/ab/summary.txt
done
