#!/bin/bash
# Round 6, session 5: the listener guard's RCCL probe, then the whole GPU
# suite, smoke and the driver's command on this tree.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
step r6_lg_probe 200 python tools/probe/listen_guard_probe.py
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
