# Round 2: 256x256 edge mode with ragged K + remainder strips
source tools/gpu_steps.sh
export TMPDIR=/tmp
step kernel_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm"
step gemm_edge 300 python tools/gemm_edge_bench.py
