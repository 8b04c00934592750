# Round 2 session 3: executor spawned with GPU_MAX_HW_QUEUES=2 by default; vs BEE_EXECUTOR_HW_QUEUES=4, interleaved; sandbox GPU tests
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2 3; do
step d_$i 300 python bench.py --steps 600 --materialized-steps 0
step e4_$i 300 env BEE_EXECUTOR_HW_QUEUES=4 python bench.py --steps 600 --materialized-steps 0
done
