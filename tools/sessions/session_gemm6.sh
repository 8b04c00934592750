source tools/gpu_steps.sh
export TMPDIR=/tmp
step gemm_lab_group 400 python -u tools/gemm_lab.py --variants 11 16 17 18 --rounds 7 --reps 20 --repeats 4
