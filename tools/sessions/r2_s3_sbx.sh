# Round 2 session 3: where a sandbox's CPU goes (pooled phase stamps through a live service; standalone lifecycle probe)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 12
step workercost 300 python tools/probe/worker_cost.py --n 200
