# Round 2 session 3: the zygote's C bootstrap per step (BEE_DEBUG_BOOT) + pooled-phase stamps
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 12
