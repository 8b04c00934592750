#!/bin/bash
# Round 6, session 22: memory-side counters (L2 hit rate, VMEM latency, TA
# busy) of the f64 GEMM against torch at 2048^3 and 1536^3.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_*
for n in 2048 1536; do
  PASSES="1 4" step pmc_f64_$n 300 bash tools/gemm_fp_pmc.sh float64 $n
  { echo "## float64 $n"; python3 tools/gemm_fp_pmc.py gpurun_out float64 $n; echo; } >> gpurun_out/pmc_tables.md
  rm -rf gpurun_out/pmc_float64_${n}_*
done
