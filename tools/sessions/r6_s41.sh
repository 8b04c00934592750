#!/bin/bash
# Round 6, session 41: grids of 1-1.5 64 x 64 tiles per CU (1152^3, 1216^3):
# the 64 x 64 two-K-group split (default) vs 64 x 32 tiles, one group.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="1088 1152 1216" step r6_sweep_ks2edge 600 bash tools/gemm_fp_sweep.sh "def" "n32 BK_GEMM_FP_KS=1 BK_GEMM_FP_BN=32" "n64 BK_GEMM_FP_KS=1 BK_GEMM_FP_BN=64" \
  "defb" "n32b BK_GEMM_FP_KS=1 BK_GEMM_FP_BN=32"
