source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step b_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_long 300 python bench.py --gpus 1
step b_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
