export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --extra-systems= > gpurun_out/r05v/bench_$i.json 2> gpurun_out/r05v/bench_$i.err || exit 1
  python3 tools/bench_summary.py gpurun_out/r05v/bench_$i.json
  python3 -c "import json;d=json.loads(open('gpurun_out/r05v/bench_$i.json').read().strip().splitlines()[-1]);print(d['segments']['rates'], d['roofline']['kernel_ms'], d['ms_per_step'])"
done
