#!/bin/bash
# Round 6, session 26: counter passes of the buffer-load 64 x 64 kernels
# against torch at 2048^3 (f32 and f64), the sweep of the final launch choice.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_*
step r6_gemm_tests 400 python -u -m pytest tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -q "passed" gpurun_out/r6_gemm_tests.log && ! grep -q "failed\|error" gpurun_out/r6_gemm_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096 8192" step r6_sweep_final 600 bash tools/gemm_fp_sweep.sh "final"
for dt in float32 float64; do
  PASSES="1 2 3 4" step pmc_${dt}_2048 400 bash tools/gemm_fp_pmc.sh $dt 2048
  { echo "## $dt 2048 (buffer loads)"; python3 tools/gemm_fp_pmc.py gpurun_out $dt 2048 bk torch; echo; } >> gpurun_out/pmc_tables.md
  rm -rf gpurun_out/pmc_${dt}_2048_*
done
