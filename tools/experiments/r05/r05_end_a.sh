export TMPDIR=/tmp
mkdir -p gpurun_out/r05e
source tools/gpu_step.sh
step 600 gpurun_out/r05e/gpu_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/r05e/gpu_all.log
step 200 gpurun_out/r05e/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 gpurun_out/r05e/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05e/bench_full.json 2> gpurun_out/r05e/bench_full.err
echo "bench rc=$?"
python3 tools/bench_summary.py gpurun_out/r05e/bench_full.json
