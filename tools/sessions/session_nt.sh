# non-temporal streaming kernels: numerics, kernel bench, payload (both
# lowerings), sandbox tests (escapee reaper), headline bench
source tools/gpu_steps.sh
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step kbench 300 python tools/bench_kernels.py
step payload_mat 120 env BEE_LAZY_RANDOM=0 python tools/payload_direct.py --iters 20
step payload_lazy 120 python tools/payload_direct.py --iters 20
step bench 300 python bench.py --steps 100
