source tools/gpu_steps.sh
for i in 1 2 3 4; do
  step q0_$i 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1 --steps 20 --warmup 5
  step q32_$i 300 python tools/probe/affinity_ab.py --cpus 32 -- --gpus 1 --steps 20 --warmup 5
done
step q0_long 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1
step q32_long 300 python tools/probe/affinity_ab.py --cpus 32 -- --gpus 1
