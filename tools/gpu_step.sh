# Run one GPU step under its own time limit and stop the whole call after a hang / kill / fault
# (exit 124 / 137 / 134 / 139): usage  step SECONDS LOGFILE cmd...   (source this file)
step() {
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> gpurun_out/steps.txt
  case $rc in 124|137|134|139) echo "fatal rc=$rc in: $*"; exit $rc;; esac
  return 0
}
