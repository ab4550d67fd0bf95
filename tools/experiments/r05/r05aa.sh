export TMPDIR=/tmp
mkdir -p gpurun_out/r05aa
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config0 --extra-systems= --update-steps 200 > gpurun_out/r05aa/bench_$i.json 2> gpurun_out/r05aa/bench_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r05aa/bench_$i.json').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1), [round(r/1e6) for r in d['segments']['rates']], round(d['long_region']['median']/1e6,1), d['roofline']['kernel_ms'])"
done
