#!/bin/bash
# Round 6, session 33: small f32 products on the 32-deep K tile by default --
# the GEMM numerics tests, then the sweep (default vs the 16-deep tile).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
DTYPES=float32 SIZES="1024 1536 2048" step r6_sweep_bk 600 bash tools/gemm_fp_sweep.sh "def" "bk16 BK_GEMM_FP_BK=16" "defb" "bk16b BK_GEMM_FP_BK=16"
