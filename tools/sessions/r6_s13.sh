#!/bin/bash
# Round 6, session 13: counters of the reworked f64 / f32 GEMM against torch
# (f64 2048^3, f32 1024^3 / 2048^3), and tile variants at f64 4096 / 8192.
# (counter databases are tabulated on the box and dropped: gpurun_out <= 64 MiB)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
for x in "float64 2048" "float32 1024" "float32 2048"; do
  set -- $x
  PASSES="1 2 3" step pmc_$1_$2 300 bash tools/gemm_fp_pmc.sh $1 $2
  { echo "## $1 $2"; python3 tools/gemm_fp_pmc.py gpurun_out $1 $2; echo; } >> gpurun_out/pmc_tables.md
  rm -rf gpurun_out/pmc_$1_$2_*
done
DTYPES=float64 SIZES="4096 8192" ROUNDS=3 step fp_sweep 900 bash tools/gemm_fp_sweep.sh "cur" "bn64 BK_GEMM_FP_BN=64" "bm64 BK_GEMM_FP_BM=64 BK_GEMM_FP_BN=64"
