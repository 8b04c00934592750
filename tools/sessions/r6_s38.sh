#!/bin/bash
# Round 6, session 38: products of at most half a CU's worth of 64 x 64
# tiles (<= 512^3) on 64 x 32 tiles with two K groups (twice the
# workgroups) against the 64 x 64 split (BK_GEMM_FP_TINY=0).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
SIZES="256 384 512 640 768" step r6_sweep_tiny 600 bash tools/gemm_fp_sweep.sh "tiny" "old BK_GEMM_FP_TINY=0" "tinyb" "oldb BK_GEMM_FP_TINY=0"
