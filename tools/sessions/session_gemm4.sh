source tools/gpu_steps.sh
step gemm_lab4 400 python tools/gemm_lab.py --variants 0 1 --no-check --rounds 9
