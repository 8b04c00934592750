source tools/gpu_steps.sh
for i in 1 2 3; do
  BEE_BENCH_TRACE=gpurun_out/trace_s10_short$i.json step b10_short$i 240 python bench.py --gpus 1 --steps 20 --warmup 5
done
step b10_default 300 python bench.py --gpus 1
