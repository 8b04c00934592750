source tools/gpu_steps.sh
step stamps 120 python tools/gemm_lab.py --stamps
step lab7 300 python tools/gemm_lab.py --variants 11 35 36 --rounds 9 --reps 20
