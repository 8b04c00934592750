#!/bin/bash
# Round 6, session 16: f32 fragments 4 k per lane (ds_read_b128 A reads, permuted
# k order, conflict-free pitches) -- tests, sweep, f32 counters.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
DTYPES=float32 SIZES="1024 1536 2048 3072 4096" EXTRA="--transposes" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "vk" "vk_rs1 BK_GEMM_FP_RS=1" "vk_bk32 BK_GEMM_FP_BK=32"
IMPLS=bk PASSES="1 2 3" step pmc_f32 300 bash tools/gemm_fp_pmc.sh float32 2048
{ echo "## float32 2048"; python3 tools/gemm_fp_pmc.py gpurun_out float32 2048 bk; } >> gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_float32_2048_*
