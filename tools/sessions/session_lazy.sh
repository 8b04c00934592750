source tools/gpu_steps.sh
step hello_eager 300 python bench.py --workload hello --steps 100
step hello_lazy 300 env BEE_BROKER_LAZY=1 python bench.py --workload hello --steps 100
step numpy_eager 300 python bench.py --steps 100
step numpy_lazy 300 env BEE_BROKER_LAZY=1 python bench.py --steps 100
step hello_eager2 300 python bench.py --workload hello --steps 100
step numpy_lazy2 300 env BEE_BROKER_LAZY=1 python bench.py --steps 100
