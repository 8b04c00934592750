# sandbox GPU tests + burst/sustained bench + CPU per request by role
source tools/gpu_steps.sh
step sbtests 400 python -u -m pytest tests/test_sandbox_gpu.py tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_a 300 python bench.py --steps 30
step bench_long 300 python bench.py --steps 300
export CPU_BD_DELAY=6 CPU_BD_WINDOW=4
step cpu_bd 300 python tools/cpu_breakdown.py --steps 3000 --warmup 3
step kbench 300 python tools/bench_kernels.py
step suite 900 python tools/bench_suite.py --out gpurun_out/bench_suite.jsonl
