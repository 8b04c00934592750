#!/bin/bash
# Helper for gpurun sessions: `step NAME TIMEOUT cmd...` runs one GPU step under
# its own time limit, logs to gpurun_out/NAME.log, and ends the whole session on
# a fault-like exit (timeout 124/137, abort 134, segfault 139) so nothing else
# touches a GPU that may be in a bad state.  Ordinary failures (rc 1, e.g. a
# failing test) do not stop later steps.
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc wall=$(awk "BEGIN{print $(date +%s.%N) - $t0}")s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "[step] fatal rc=$rc, ending session"; exit $rc; fi
  return 0
}
