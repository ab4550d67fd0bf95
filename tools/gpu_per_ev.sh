# car_park PER B=4096: device- vs system-scope pipeline events (rates + a short trace of each)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/perev
mkdir -p $D
for v in dev sys; do
  if [ $v = sys ]; then export CACTO_EVENT_SYSFENCE=1; else unset CACTO_EVENT_SYSFENCE; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 1000 --extra-systems car_park > $D/b$v.json 2> $D/b$v.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$v.json').read().strip().splitlines()[-1])
print('$v', {s: {k: round(v['value']) for k, v in e['critic_updates'].items()} for s, e in d['extra_systems'].items()})
" >> $D/summary.txt
  timeout -k 10 300 rocprofv3 --kernel-trace -d $D/t$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 300 --extra-systems car_park > $D/p$v.json 2> $D/p$v.err &&
  python3 tools/timeline.py $D/t$v/run_results.db k_ 30 200 > $D/timeline_$v.txt && rm -rf $D/t$v
done
