#!/bin/bash
# Round 6, session 27: f32 [m][k] LDS rows padded by 8 B instead of 16 B
# (this build) against the 16-B build (ablib/base.so), same box.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_*
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
DTYPES=float32 SIZES="1024 1536 2048 3072 4096 8192" step r6_sweep_pitch 600 bash tools/gemm_fp_sweep.sh "pad8" "pad16 BEE_KERNEL_LIB=ablib/base.so" "pad8b" "pad16b BEE_KERNEL_LIB=ablib/base.so"
IMPLS=bk PASSES="1 3" step pmc_f32 300 bash tools/gemm_fp_pmc.sh float32 2048
{ echo "## float32 2048 (8-B padded rows)"; python3 tools/gemm_fp_pmc.py gpurun_out float32 2048 bk; echo; } >> gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_float32_2048_*
