source tools/gpu_steps.sh
step stamps4 120 python tools/gemm_lab.py --stamps
step lab10 300 python tools/gemm_lab.py --variants 37 41 --rounds 9 --reps 20
