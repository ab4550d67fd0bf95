export TMPDIR=/tmp
mkdir -p gpurun_out/r05fa
source tools/gpu_step.sh
step 900 gpurun_out/r05fa/gpu_all.log python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
tail -3 gpurun_out/r05fa/gpu_all.log
step 200 gpurun_out/r05fa/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 gpurun_out/r05fa/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05fa/bench_full.json 2> gpurun_out/r05fa/bench_full.err
echo "bench rc=$?"
python3 tools/bench_summary.py gpurun_out/r05fa/bench_full.json
