#!/bin/bash
# Round 6, session 23: the f64 / f32 GEMM's branch-free buffer-descriptor
# loads (BK_GEMM_FP_BUF, out-of-range reads return zero, no edge-tile loop):
# the GEMM and offload numerics tests, then the sweep against the guarded
# build (BK_GEMM_FP_BUF=0) and torch.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_buf_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
SIZES="1024 1536 2048 3072 4096" step r6_buf_sweep 600 bash tools/gemm_fp_sweep.sh "buf" "nobuf BK_GEMM_FP_BUF=0"
