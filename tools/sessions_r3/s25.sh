source tools/gpu_steps.sh
step stamps3 120 python tools/gemm_lab.py --stamps
