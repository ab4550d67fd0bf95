bash tools/prof_round.sh r05
echo "prof rc=$?"
ls gpurun_out/prof_r05
