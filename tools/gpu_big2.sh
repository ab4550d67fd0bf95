# large-batch update loop: device-scope vs system-scope events; tests; one kernel trace
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/big2
mkdir -p $D
for v in dev sys; do
  if [ $v = sys ]; then export CACTO_EVENT_SYSFENCE=1; else unset CACTO_EVENT_SYSFENCE; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 4096 --update-steps 500 > $D/b$v.json 2> $D/b$v.err || exit 1
  python3 -c "
import json
d=json.loads(open('$D/b$v.json').read().strip().splitlines()[-1])
print('$v DI B=4096 %.0f' % d['critic_updates']['B=4096']['value'], {s: {k: round(v['value']) for k, v in e['critic_updates'].items()} for s, e in d['extra_systems'].items()})
" >> $D/summary.txt
done
unset CACTO_EVENT_SYSFENCE
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches 4096 --update-steps 500 --extra-systems "" > $D/prof.log 2>&1
