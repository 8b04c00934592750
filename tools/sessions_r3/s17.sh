source tools/gpu_steps.sh
for i in 1 2 3; do
  step sw_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  APP_STARTUP_SELF_WARM_EXECUTIONS=0 step nosw_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
step sw_long 300 python bench.py --gpus 1
