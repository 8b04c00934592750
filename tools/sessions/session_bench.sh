source tools/gpu_steps.sh
step bench 300 python bench.py --steps 100
