#!/bin/bash
# Round 6, session 3: the whole GPU suite and smoke on this tree (listener
# guard, trusted prefault, GPU timing, tight GEMM bounds), the driver's
# command, and the headline with the listener guard on vs off (600 steps x 2).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/cpu_ab.jsonl
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step r6_guard_ab 1100 bash tools/cpu_ab.sh 600 2 guard noguard=APP_SANDBOX_LISTEN_GUARD=0
