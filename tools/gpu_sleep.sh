# team-barrier poll sleep (k_rollout_tt, DI): s_sleep 1 (default) / 0 / 2, DI rollout rates twice each
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/sl
mkdir -p $D
for r in a b; do
for v in 1 0 2; do
  if [ $v = 1 ]; then L=cacto_amd/libcacto_hip.so; else L=cacto_amd/libcacto_hip_sl$v.so; fi
  CACTO_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 500 --batches "" --update-steps 20 --extra-systems car_park > $D/b$v$r.json 2> $D/b$v$r.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$v$r.json').read().strip().splitlines()[-1])
print('sleep $v $r DI %.1f M long %.1f M kern %.4f ms' % (d['value']/1e6, d['long_region']['median']/1e6, d['roofline']['kernel_ms']), 'car_park long %.1f M' % (d['extra_systems']['car_park']['long_region']['median']/1e6))
" >> $D/summary.txt
done
done
