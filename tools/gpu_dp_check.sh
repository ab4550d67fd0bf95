# all GPU tests, then a 2-rank rehearsal of the multi-GPU bench on the one device (gloo)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 &&
CACTO_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --update-steps 100 --no-cpu-baseline --no-diagnostics --no-config0 > gpurun_out/bench_dp2.json 2> gpurun_out/bench_dp2.err
