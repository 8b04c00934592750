source tools/gpu_steps.sh
step b_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_long 300 python bench.py --gpus 1
