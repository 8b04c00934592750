#!/bin/bash
# Round 6, session 20: the tree after the f64 / f32 GEMM work -- the whole GPU
# suite, smoke, the driver's bench command; then a shape sweep for the
# launcher's choice at the sizes still short of torch.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/gemm_fp_sweep.jsonl
step r6_gputests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r6_bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
DTYPES=float64 SIZES="1536 2048" ROUNDS=3 step sweep64 600 bash tools/gemm_fp_sweep.sh "cur" \
  "bn32 BK_GEMM_FP_BN=32" "ks2 BK_GEMM_FP_BN=64 BK_GEMM_FP_KS=2" "bm128 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=64"
DTYPES=float32 SIZES="1536 2048" ROUNDS=3 step sweep32 600 bash tools/gemm_fp_sweep.sh "cur" \
  "bn32 BK_GEMM_FP_BM=64 BK_GEMM_FP_BN=32" "bn64 BK_GEMM_FP_BM=64 BK_GEMM_FP_BN=64" "ks2 BK_GEMM_FP_BM=64 BK_GEMM_FP_BN=64 BK_GEMM_FP_KS=2" \
  "bm128n64 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=64" "bm128n128 BK_GEMM_FP_BM=128 BK_GEMM_FP_BN=128" "bk32 BK_GEMM_FP_BK=32"
