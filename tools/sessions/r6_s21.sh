#!/bin/bash
# Round 6, session 21: the tree with the listener-guard fixes (no blocking
# accept in the guard thread, per-sandbox cap, bounded scans) -- the RCCL
# example through the guard, the whole GPU suite, smoke, the driver's bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
step r6_lg_probe 200 python tools/probe/listen_guard_probe.py
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
