# Round 2 session 3: per-op wall time of the headline payload inside sandboxes at concurrency 1/4/8/16
source tools/gpu_steps.sh
export TMPDIR=/tmp
step breakdown 400 python tools/payload_breakdown.py
