# Round 2: [K][N] GEMM kernel (transposed LDS reads): tests + bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
step nn_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "nn or row_major or gemm_kernel_variants"
step nn_bench 300 python tools/gemm_nn_bench.py
