# Round 2: GEMM after moving edge/NN instantiations to their own TU (shipped kernel spill-free again)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step kernel_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step gemm_edge 300 python tools/gemm_edge_bench.py
step nn_bench 300 python tools/gemm_nn_bench.py
