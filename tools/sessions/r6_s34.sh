#!/bin/bash
# Round 6, session 34: two K groups on 64 x 32 tiles (twice the workgroups of
# the 64 x 64 split) for the small products; plus the new wide-ld test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=2 step r6_gemm_tests_k2n32 400 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split_k or matches_fp64 or ragged"
SIZES="768 1024 1280 1536" step r6_sweep_k2n32 600 bash tools/gemm_fp_sweep.sh "def" "k2n32 BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=2" "defb" "k2n32b BK_GEMM_FP_BN=32 BK_GEMM_FP_KS=2"
