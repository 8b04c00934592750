source tools/gpu_steps.sh
step gputests32 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2 3; do
  step b32_nosite_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  BEE_NANO_NO_SITE=0 step b32_site_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
step b32_nosite_600 300 python bench.py --gpus 1
BEE_NANO_NO_SITE=0 step b32_site_600 300 python bench.py --gpus 1
step b32_fib 300 python bench.py --gpus 1 --workload fib --steps 20 --warmup 5
step b32_hello 300 python bench.py --gpus 1 --workload hello --steps 50 --warmup 5
step sbdebug32 300 python tools/probe/sandbox_debug.py --n 10
