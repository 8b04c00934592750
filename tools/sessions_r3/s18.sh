source tools/gpu_steps.sh
for i in 1 2 3; do
  APP_STARTUP_SELF_WARM_EXECUTIONS=3072 step sw3k_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step sw1k_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
