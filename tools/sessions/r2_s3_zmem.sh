# Round 2 session 3: where a minimal zygote's small-page anonymous memory lives (per mapping)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 2
