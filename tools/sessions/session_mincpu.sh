source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step hello 300 python bench.py --workload hello --steps 100
step numpy 300 python bench.py --steps 100
step hello2 300 python bench.py --workload hello --steps 100
step numpy2 300 python bench.py --steps 100
