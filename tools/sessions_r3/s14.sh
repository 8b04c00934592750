source tools/gpu_steps.sh
for i in 1 2; do
  step n0_$i 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1 --steps 20 --warmup 5
  step p24_$i 300 python tools/probe/affinity_ab.py --cpus 24 -- --gpus 1 --steps 20 --warmup 5
  step s32_$i 300 python tools/probe/affinity_ab.py --cpus 32 --smt -- --gpus 1 --steps 20 --warmup 5
  step p32_$i 300 python tools/probe/affinity_ab.py --cpus 32 -- --gpus 1 --steps 20 --warmup 5
done
step n0_long 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1
step p24_long 300 python tools/probe/affinity_ab.py --cpus 24 -- --gpus 1
step s32_long 300 python tools/probe/affinity_ab.py --cpus 32 --smt -- --gpus 1
step p32_long 300 python tools/probe/affinity_ab.py --cpus 32 -- --gpus 1
