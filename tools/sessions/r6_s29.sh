#!/bin/bash
# Round 6, session 29: where the next K tile is staged (LDS stores + global
# loads) inside the iteration: top (in-tree build) vs after MFMA step 1 / 2
# (ablib/x1.so, ablib/x2.so built with -DBK_FP_STORE_AT=1 / 2).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
for v in x1 x2; do
  BEE_KERNEL_LIB=ablib/$v.so step r6_tests_$v 300 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
  grep -q "passed" gpurun_out/r6_tests_$v.log && ! grep -q "failed\|error" gpurun_out/r6_tests_$v.log || { echo "tests failed"; exit 1; }
done
SIZES="1536 2048 3072 4096" step r6_sweep_storeat 600 bash tools/gemm_fp_sweep.sh "x0" "x1 BEE_KERNEL_LIB=ablib/x1.so" "x2 BEE_KERNEL_LIB=ablib/x2.so" \
  "x0b" "x1b BEE_KERNEL_LIB=ablib/x1.so" "x2b BEE_KERNEL_LIB=ablib/x2.so"
