source tools/gpu_steps.sh
step gputests31 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2 3; do
  step b31_nano_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  APP_NANO_WORKERS_PER_GPU_TARGET=0 step b31_min_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
step b31_nano_600 300 python bench.py --gpus 1
APP_NANO_WORKERS_PER_GPU_TARGET=0 step b31_min_600 300 python bench.py --gpus 1
