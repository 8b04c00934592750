#!/bin/bash
# Round 6, session 42: two K groups only up to one 64 x 64 tile per CU --
# GEMM tests, the sweep around the boundary, then the final tree again
# (the review's GEMM command, the GPU suite, smoke, the driver's bench, 600
# steps).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="960 1024 1088 1152 1216 1280" step r6_sweep_ks2cap 600 bash tools/gemm_fp_sweep.sh "cap"
step r6_fp_final 600 python tools/gemm_fp_bench.py --sizes 1024 1536 2048 3072 4096 8192 --rounds 3 --x6 --transposes
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
step r6_bench_600 600 python bench.py --gpus 1 --steps 600 --warmup 50
