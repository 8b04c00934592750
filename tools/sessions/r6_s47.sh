#!/bin/bash
# Round 6, session 47: tile-row groups of 2 / 1 (ablib builds) against 4
# (in-tree) at the larger sizes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
SIZES="2048 4096 8192" step r6_sweep_group2 600 bash tools/gemm_fp_sweep.sh "g4" "g2 BEE_KERNEL_LIB=ablib/g2.so" "g1 BEE_KERNEL_LIB=ablib/g1.so" \
  "g4b" "g2b BEE_KERNEL_LIB=ablib/g2.so" "g1b BEE_KERNEL_LIB=ablib/g1.so"
