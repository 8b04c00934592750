#!/bin/bash
# Round 6, session 46: the final tree (tile groups of 4) -- the review's GEMM
# command, the whole GPU suite, smoke, the driver's bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
step r6_fp_final 600 python tools/gemm_fp_bench.py --sizes 1024 1536 2048 3072 4096 8192 --rounds 3 --x6 --transposes
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
