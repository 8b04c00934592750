source tools/gpu_steps.sh
step sbdebug 300 python tools/probe/sandbox_debug.py --n 12
