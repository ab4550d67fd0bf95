# multi-workgroup PER sampling / subtree priority update: PER parity tests on the default selection and
# with every batch forced onto the new kernels, then the car_park PER update rates
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/per
mkdir -p $D
T="tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_update_parity.py tests/test_gpu_dp.py tests/test_gpu_main_loop.py tests/test_gpu_graph.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
CACTO_PER_MW_MIN=1 timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread -k "per or PER or Per or buffer or main_loop" > $D/tests_mw1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config0 --no-diagnostics --long-steps 0 --batches "" --update-steps 500 --extra-systems car_park > $D/b.json 2> $D/b.err || exit 1
python3 -c "
import json
d=json.loads(open('$D/b.json').read().strip().splitlines()[-1])
print({s: {k: round(v['value']) for k, v in e['critic_updates'].items()} for s, e in d['extra_systems'].items()})
" >> $D/summary.txt
