# Round 2 session 3: matmul(a, b) picks the [K][N] kernel by M (BEE_GEMM_NN=auto); GEMM GPU tests
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gemmtests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or matmul" --timeout 120 --timeout-method thread -p no:cacheprovider
