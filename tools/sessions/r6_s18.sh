#!/bin/bash
# Round 6, session 18: two-stage register pipeline with its global loads as
# inline asm (each LDS store waits for its own stage only) -- tests, sweep,
# f64 counters.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
step fp_tests 300 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096 8192" ROUNDS=3 EXTRA="--transposes" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "async"
IMPLS=bk PASSES="1 2 3" step pmc_f64 300 bash tools/gemm_fp_pmc.sh float64 2048
{ echo "## float64 2048 (async loads)"; python3 tools/gemm_fp_pmc.py gpurun_out float64 2048 bk; } >> gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_float64_2048_*
