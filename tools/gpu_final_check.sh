# smoke() + a 2-rank rehearsal of the multi-GPU bench on one GPU (gloo collectives, ranks share the device)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
CACTO_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-diagnostics --update-steps 10 > gpurun_out/bench_dp2.json 2> gpurun_out/bench_dp2.err
