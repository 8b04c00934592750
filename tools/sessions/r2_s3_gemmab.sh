# Round 2 session 3: TN GEMM vs hipBLASLt, current build (interleaved rounds, one process)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gemmab 300 python tools/gemm_ab.py --rounds 5 --reps 20
