#!/bin/bash
# Round 6, session 30: the register-slot loop with both steps unconditional
# and an odd last step peeled (ablib/pair.so) against the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
BEE_KERNEL_LIB=ablib/pair.so step r6_tests_pair 300 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_tests_pair.log && ! grep -q "failed\|error" gpurun_out/r6_tests_pair.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096" step r6_sweep_pair 600 bash tools/gemm_fp_sweep.sh "head" "pair BEE_KERNEL_LIB=ablib/pair.so" "headb" "pairb BEE_KERNEL_LIB=ablib/pair.so"
