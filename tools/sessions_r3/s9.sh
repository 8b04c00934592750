source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
BEE_BENCH_TRACE=gpurun_out/trace_s9_short1.json step b9_short1 240 python bench.py --gpus 1 --steps 20 --warmup 5
step b9_default 300 python bench.py --gpus 1
BEE_BENCH_TRACE=gpurun_out/trace_s9_short2.json step b9_short2 240 python bench.py --gpus 1 --steps 20 --warmup 5
PROF_DIR=gpurun_out/prof_s9 step prof9 300 bash tools/prof_served.sh 300
