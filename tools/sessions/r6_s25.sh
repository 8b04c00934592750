#!/bin/bash
# Round 6, session 25: 64-row tiles for f32 too (the 128-row ones dropped
# from the launch choice); the numerics tests, then the default against the
# guarded build and the 32-deep f32 K tile.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
SIZES="1024 1536 2048 3072 4096 8192" step r6_sweep_64 900 bash tools/gemm_fp_sweep.sh "def" "nobuf BK_GEMM_FP_BUF=0" "bk32 BK_GEMM_FP_BK=32"
