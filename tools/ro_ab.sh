# Rollout kernel A/B of library variants: tools/ro_sched.py per variant, alternated twice.
# Usage: bash tools/ro_ab.sh SYSTEM R "g,w ..." lib1.so lib2.so ...
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
SYS=$1; R=$2; SCH=$3; shift 3
for rep in 1 2; do
  for L in "$@"; do
    echo "== $(basename $L) rep $rep" >> gpurun_out/ab/ro_ab.log
    CACTO_HIP_LIB=$L timeout -k 10 120 python -u tools/ro_sched.py $SYS $R "$SCH" >> gpurun_out/ab/ro_ab.log 2>&1
  done
done
