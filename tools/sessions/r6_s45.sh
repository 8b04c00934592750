#!/bin/bash
# Round 6, session 45: the tile order's group of tile rows (4 / 16, ablib
# builds) against 8 (in-tree) at the larger sizes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="2048 4096 8192" step r6_sweep_group 600 bash tools/gemm_fp_sweep.sh "g8" "g4 BEE_KERNEL_LIB=ablib/g4.so" "g16 BEE_KERNEL_LIB=ablib/g16.so" \
  "g8b" "g4b BEE_KERNEL_LIB=ablib/g4.so" "g16b BEE_KERNEL_LIB=ablib/g16.so"
