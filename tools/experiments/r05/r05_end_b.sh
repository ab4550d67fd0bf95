export TMPDIR=/tmp
timeout -k 10 1100 bash tools/prof_round.sh r05 > gpurun_out/prof_r05.log 2>&1
echo "prof rc=$?"
ls gpurun_out/prof_r05
