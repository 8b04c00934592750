#!/bin/bash
# Round 6, session 14: f64 / f32 GEMM with conflict-free f32 rows and no
# ds_read2 pairing, f64 on 64 x 64 tiles throughout -- tests, sweep, counters.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
rm -f gpurun_out/gemm_fp_sweep.jsonl gpurun_out/pmc_tables.md
rm -rf gpurun_out/pmc_* gpurun_out/trace_*
step fp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_fp_gpu.py tests/test_offload_gpu.py
grep -q "passed" gpurun_out/fp_tests.log && ! grep -q "failed\|error" gpurun_out/fp_tests.log || { echo "tests failed"; exit 1; }
SIZES="1024 1536 2048 3072 4096" EXTRA="--transposes" step fp_sweep 900 bash tools/gemm_fp_sweep.sh "v3"
for x in "float64 2048" "float32 2048"; do
  set -- $x
  IMPLS=bk PASSES="1 2 3" step pmc_$1_$2 300 bash tools/gemm_fp_pmc.sh $1 $2
  { echo "## $1 $2"; python3 tools/gemm_fp_pmc.py gpurun_out $1 $2 bk; echo; } >> gpurun_out/pmc_tables.md
  rm -rf gpurun_out/pmc_$1_$2_*
done
