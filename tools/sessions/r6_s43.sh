#!/bin/bash
# Round 6, session 43: the buffer descriptor's range capped at 2^31 - 1 (a
# panel of 4 GiB and more used to wrap) -- the GEMM tests with the 4.5 GB
# operand, the offload tests, smoke.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
