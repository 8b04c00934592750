#!/bin/bash
# rocprofv3 kernel trace of the served path: the executor daemon (kernel
# broker) under the profiler, driven with N Execute requests of the headline
# payload, then stopped with SIGTERM so the profiler flushes at exit.
#   bash tools/prof_served.sh [N]       (from the repo root, on the GPU box)
set -u
N=${1:-200}
D=$(mktemp -d /tmp/bee-prof-XXXXXX)
mkdir -p gpurun_out
mapfile -t CMD < <(python tools/prof_served.py cmd "$D")
export BEE_PROFILE_DAEMON_ONLY=1 TMPDIR=/tmp
# PROF_FLAGS: what to trace (default kernels + the broker's roctx ranges;
# e.g. "--hip-runtime-trace --marker-trace" for host time per HIP call);
# PROF_DIR: output directory under gpurun_out
FLAGS=${PROF_FLAGS:---kernel-trace --marker-trace --stats}
OUT=${PROF_DIR:-gpurun_out/prof_served}
# shellcheck disable=SC2086
timeout -k 10 150 rocprofv3 $FLAGS -d "$OUT" -o run -- "${CMD[@]}" \
  > gpurun_out/prof_served_daemon.log 2>&1 &
ROC=$!
timeout -k 10 180 python tools/prof_served.py drive "$D" --n "$N"
RC=$?
timeout -k 5 30 python tools/prof_served.py shutdown "$D"
wait "$ROC"
echo "[prof_served] drive rc=$RC profiler rc=$?"
rm -rf "$D"
exit $RC
