source tools/gpu_steps.sh
for i in 1 2; do
  step w5_$i 240 python bench.py --gpus 1 --steps 20 --warmup 5
  step w50_$i 240 python bench.py --gpus 1 --steps 20 --warmup 50
  step w200_$i 240 python bench.py --gpus 1 --steps 20 --warmup 200
done
