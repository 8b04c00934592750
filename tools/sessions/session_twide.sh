source tools/gpu_steps.sh
export TMPDIR=/tmp
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step stests 300 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
