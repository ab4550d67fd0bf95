# manipulator B = 8192 update loop kernel timeline with the wait kernel
set -e
export TMPDIR=/tmp
D=gpurun_out/r05ae
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run -- python3 bench.py --steps 2 --warmup 1 --update-steps 300 --batches 128 --extra-systems manipulator --no-cpu-baseline --no-diagnostics --no-config0 --long-steps 0 > $D/b.json 2> $D/b.err
python3 tools/timeline.py $D/t/run_results.db k_ 40 200 > $D/timeline.txt
rm -rf $D/t
cat $D/timeline.txt
