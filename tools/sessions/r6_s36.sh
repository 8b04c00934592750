#!/bin/bash
# Round 6, session 36: 64 x 32 vs 64 x 64 by how evenly the tiles spread
# over the CUs, the f32 K tile tied to the shape -- tests, then the sweep
# over the standard and in-between sizes (default vs the previous rule's
# choice forced by env).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1280 1536 1792 2048 2560 3072" step r6_sweep_fill 600 bash tools/gemm_fp_sweep.sh "fill" "fillb"
