source tools/gpu_steps.sh
export TMPDIR=/tmp
step gemmab42 300 python tools/gemm_ab.py --rounds 5
