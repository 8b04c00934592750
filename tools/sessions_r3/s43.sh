source tools/gpu_steps.sh
for i in 1 2 3; do
  step b43_lg1_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step b43_lg2_short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --clients-per-loadgen 4
done
step b43_lg1_600 300 python bench.py --gpus 1
step b43_lg2_600 300 python bench.py --gpus 1 --clients-per-loadgen 4
