#!/bin/bash
# Round 6, session 15: XCD order for any tile count, f64 on 64 x 64 tiles
# throughout, the f64 32-deep K tile as a variant.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096 8192" ROUNDS=3 step fp_sweep 900 bash tools/gemm_fp_sweep.sh "v4"
DTYPES=float64 SIZES="1024 1536 2048 3072" step fp_sweep2 600 bash tools/gemm_fp_sweep.sh "bk32 BK_GEMM_FP_BK=32" "bk32rs1 BK_GEMM_FP_BK=32 BK_GEMM_FP_RS=1"
