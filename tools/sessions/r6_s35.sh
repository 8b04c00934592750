#!/bin/bash
# Round 6, session 35: the launch choice at in-between sizes (1280, 1792,
# 2560): default vs 16-deep f32 tile, 64 x 64 and 64 x 32 tiles.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="1280 1792 2560" step r6_sweep_mid 600 bash tools/gemm_fp_sweep.sh "def" "bk16 BK_GEMM_FP_BK=16" "bn64 BK_GEMM_FP_BN=64" \
  "bn64k16 BK_GEMM_FP_BN=64 BK_GEMM_FP_BK=16" "bn32 BK_GEMM_FP_BN=32" "bn32k16 BK_GEMM_FP_BN=32 BK_GEMM_FP_BK=16"
