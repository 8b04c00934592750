source tools/gpu_steps.sh
export TMPDIR=/tmp
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step payload_direct 120 python tools/payload_direct.py --iters 20
step prof_payload2 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_payload2 -o run -- python3 tools/payload_direct.py --iters 20
step bench 300 python bench.py
