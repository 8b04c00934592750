source tools/gpu_steps.sh
for i in 1 2 3; do
  step pin_$i 240 python bench.py --gpus 1 --steps 20 --warmup 5
  APP_CPU_QUOTA_PIN_FACTOR=0 step nopin_$i 240 python bench.py --gpus 1 --steps 20 --warmup 5
done
step pin_long 300 python bench.py --gpus 1
APP_CPU_QUOTA_PIN_FACTOR=0 step nopin_long 300 python bench.py --gpus 1
