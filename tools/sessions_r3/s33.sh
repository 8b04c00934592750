source tools/gpu_steps.sh
for i in 1 2 3; do
  step b33_default_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  BEE_NANO_NO_SITE=0 step b33_site_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  BEE_PRECOMPILE=0 step b33_nopre_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
step b33_default_600 300 python bench.py --gpus 1
BEE_PRECOMPILE=0 step b33_nopre_600 300 python bench.py --gpus 1
step sbdebug33 300 python tools/probe/sandbox_debug.py --n 10
step gputests33 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
