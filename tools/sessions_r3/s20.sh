source tools/gpu_steps.sh
step lab6 300 python tools/gemm_lab.py --variants 11 29 30 31 --rounds 9 --reps 20
