#!/bin/bash
# Round 6, session 19: the final f64 / f32 GEMM -- its tests (NaN-padded
# edges) and the review's command (tools/gemm_fp_bench.py, sizes 1024..8192,
# 3 rounds, with the f32 split) for profiles/r6_gemm_fp_final.jsonl.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
step fp_tests 300 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
step fp_final 900 python tools/gemm_fp_bench.py --sizes 1024 1536 2048 3072 4096 8192 --rounds 3 --x6 --transposes
