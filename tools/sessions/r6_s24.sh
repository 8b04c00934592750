#!/bin/bash
# Round 6, session 24: tile shapes again with the buffer-load kernels (their
# lower register peak changes how many workgroups a CU holds).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="1024 1536 2048 3072 4096" DTYPES=float64 step r6_shape_f64 600 bash tools/gemm_fp_sweep.sh "def" \
  "bn64 BK_GEMM_FP_BN=64" "m128x64 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=64" "ks1 BK_GEMM_FP_KS=1" "rs1 BK_GEMM_FP_RS=1" "bk32 BK_GEMM_FP_BK=32"
SIZES="1024 1536 2048 3072 4096" DTYPES=float32 step r6_shape_f32 600 bash tools/gemm_fp_sweep.sh "def" \
  "m128x64 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=64" "m128x128 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=128" "m64x64 BK_GEMM_FP_BM=64 BK_GEMM_FP_BN=64" \
  "ks1 BK_GEMM_FP_KS=1" "rs1 BK_GEMM_FP_RS=1" "bk32 BK_GEMM_FP_BK=32"
