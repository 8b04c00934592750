source tools/gpu_steps.sh
step stamps2 120 python tools/gemm_lab.py --stamps
step lab8 300 python tools/gemm_lab.py --variants 11 37 --rounds 9 --reps 20
