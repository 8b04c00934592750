source tools/gpu_steps.sh
step lab9 300 python tools/gemm_lab.py --variants 11 37 39 --rounds 9 --reps 20
step kern_tests 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step gemm_ab2 300 python tools/gemm_ab.py --rounds 7
