# counters list + the default bench line (new measurement layout)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err
