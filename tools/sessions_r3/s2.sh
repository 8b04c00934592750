source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
BEE_BENCH_TRACE=gpurun_out/trace_short1.json step b_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
BEE_BENCH_TRACE=gpurun_out/trace_long.json step b_long 300 python bench.py --gpus 1 --steps 300 --warmup 5
BEE_BENCH_TRACE=gpurun_out/trace_short2.json step b_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b_default 300 python bench.py --gpus 1
