source tools/gpu_steps.sh
BEE_BENCH_TRACE=gpurun_out/trace_short1.json step b_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_default 300 python bench.py --gpus 1
BEE_BENCH_TRACE=gpurun_out/trace_short2.json step b_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
BEE_BENCH_TRACE=gpurun_out/trace_short3.json step b_short3 240 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 300 bash tools/prof_served.sh 300
