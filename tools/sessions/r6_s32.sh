#!/bin/bash
# Round 6, session 32: launch-choice variants at 1024-2048^3 on the final
# kernel (32-deep f32 K tile, 64 x 32 vs 64 x 64, one vs two K groups).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="1024 1536 2048" step r6_sweep_small 600 bash tools/gemm_fp_sweep.sh "def" "bk32 BK_GEMM_FP_BK=32" "bn32 BK_GEMM_FP_BN=32" \
  "bn64 BK_GEMM_FP_BN=64" "ks1 BK_GEMM_FP_KS=1" "defb" "bk32b BK_GEMM_FP_BK=32"
