source tools/gpu_steps.sh
step lab5 300 python tools/gemm_lab.py --variants 11 25 26 27 28 --rounds 7 --reps 20
