#!/bin/bash
# Round 6, session 28: three register stages (four K tiles of loads in
# flight) for the one-K-group buffer-load kernels, against two.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
SIZES="1536 2048 3072 4096 8192" step r6_sweep_rs3 600 bash tools/gemm_fp_sweep.sh "rs2" "rs3 BK_GEMM_FP_RS=3" "rs2b" "rs3b BK_GEMM_FP_RS=3"
