#!/bin/bash
# Round 6, session 37: buffer loads for the two-K-group kernels again, now
# that the register-slot loop keeps a slot in flight (BK_GEMM_FP_BUFKS2=1).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
BK_GEMM_FP_BUFKS2=1 step r6_gemm_tests_bufks2 400 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests_bufks2.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests_bufks2.log || { echo "tests failed"; exit 1; }
SIZES="512 768 1024" step r6_sweep_bufks2 600 bash tools/gemm_fp_sweep.sh "def" "bufks2 BK_GEMM_FP_BUFKS2=1" "defb" "bufks2b BK_GEMM_FP_BUFKS2=1"
