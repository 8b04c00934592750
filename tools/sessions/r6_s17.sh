#!/bin/bash
# Round 6, session 17: the LDS-staged f64 kernel (global -> LDS loads) --
# tests first (edges), then the f64 sweep against the register-staged kernel.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
step fp_tests 300 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
DTYPES=float64 SIZES="1024 1536 2048 3072 4096 8192" ROUNDS=3 step fp_sweep 900 bash tools/gemm_fp_sweep.sh "dma" "regs BK_GEMM_FP_DMA=0"
IMPLS=bk PASSES="1 2 3" step pmc_f64 300 bash tools/gemm_fp_pmc.sh float64 2048
{ echo "## float64 2048 (LDS-staged)"; python3 tools/gemm_fp_pmc.py gpurun_out float64 2048 bk; } >> gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_float64_2048_*
