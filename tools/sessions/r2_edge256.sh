# Round 2: 256x256 GEMM edge mode on MI355X (tests + TFLOP/s vs aligned / hipBLASLt), steady-state bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
step kernel_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm"
step gemm_edge 300 python tools/gemm_edge_bench.py
step bench_np600 300 python bench.py --steps 600
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
