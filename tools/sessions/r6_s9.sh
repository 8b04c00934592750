#!/bin/bash
# Round 6, session 9: whole-tile fragment prefetch in the small f64 / f32
# GEMM tiles -- tests, then the variant sweep.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "pf" "pf_ks1 BK_GEMM_FP_KS=1" "pf_bn32 BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=1" \
  "pf_bm64 BK_GEMM_FP_BM=64"
