#!/bin/bash
# Round 6, session 8: the f64 / f32 GEMM's two-K-group workgroups (no C
# memset, no atomics) and 64 x 32 tiles -- tests, then the variant sweep.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
step fp_sweep 900 bash tools/gemm_fp_sweep.sh "default" "ks1 BK_GEMM_FP_KS=1" "bn32 BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=1" \
  "bn32ks2 BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=2" "su4 BK_GEMM_FP_SU=4 BK_GEMM_FP_SS=2" "su8s1 BK_GEMM_FP_SU=8 BK_GEMM_FP_SS=1"
