source tools/gpu_steps.sh
step gemm_lab2 400 python tools/gemm_lab.py --variants 0 1 6 7 8
