#!/bin/bash
# Round 6, session 12: the reworked f64 / f32 GEMM (lookahead + two register
# stages on every tile but 128 x 128, partial K tile first, new shape
# choice) -- tests, then the size sweep with transposed views, and the f32
# 32-deep K tile.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096" EXTRA="--transposes --x6" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "new"
DTYPES=float32 SIZES="1024 1536 2048 3072" step fp_sweep2 600 bash tools/gemm_fp_sweep.sh "bk32 BK_GEMM_FP_BK=32" "rs1 BK_GEMM_FP_RS=1"
