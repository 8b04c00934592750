source tools/gpu_steps.sh
for i in 1 2 3; do
  step numpy_eager_$i 300 python bench.py --steps 100
  step numpy_lazy_$i 300 env BEE_BROKER_LAZY=1 python bench.py --steps 100
done
