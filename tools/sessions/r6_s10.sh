#!/bin/bash
# Round 6, session 10: f64 2048^3 counters, our 64 x 64 kernel (one and two
# register stages) against torch's 64 x 64 x 16 Tensile kernel; the RS sweep.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl
rm -rf gpurun_out/pmc_*
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
PASSES="1 2 3" step pmc_a 400 bash tools/gemm_fp_pmc.sh float64 2048
BK_GEMM_FP_RS=2 IMPLS=bk TAG=rs2 PASSES="1 2 3" step pmc_b 300 bash tools/gemm_fp_pmc.sh float64 2048
SIZES="1024 1536 2048 3072" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "rs1" "rs2 BK_GEMM_FP_RS=2" "rs2ks1 BK_GEMM_FP_RS=2 BK_GEMM_FP_KS=1"
