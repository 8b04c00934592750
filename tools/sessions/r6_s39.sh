#!/bin/bash
# Round 6, session 39: the next K tile's LDS stores and its refill loads at
# separate MFMA steps (ablib/vSL.so: stores before step S, loads before L)
# against both before step 2 (in-tree build).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
for v in v12 v23 v13; do
  BEE_KERNEL_LIB=ablib/$v.so step r6_tests_$v 300 python -u -m pytest tests/test_gemm_fp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "matches_fp64 or ragged or split_k"
  grep -q "passed" gpurun_out/r6_tests_$v.log && ! grep -q "failed\|error" gpurun_out/r6_tests_$v.log || { echo "tests failed"; exit 1; }
done
SIZES="1024 1536 2048 3072 4096" step r6_sweep_sl 600 bash tools/gemm_fp_sweep.sh "s2l2" "v12 BEE_KERNEL_LIB=ablib/v12.so" "v23 BEE_KERNEL_LIB=ablib/v23.so" "v13 BEE_KERNEL_LIB=ablib/v13.so" \
  "s2l2b" "v12b BEE_KERNEL_LIB=ablib/v12.so" "v23b BEE_KERNEL_LIB=ablib/v23.so" "v13b BEE_KERNEL_LIB=ablib/v13.so"
