set -e
for o in 0 0 1 0 1 2 0 2; do
  echo "offset $o" >> gpurun_out/tt_off.log
  CACTO_TT_OFFSET=$o timeout -k 10 120 python tools/tt_smoke.py double_integrator 2>&1 | grep "sched (-1" >> gpurun_out/tt_off.log
done
