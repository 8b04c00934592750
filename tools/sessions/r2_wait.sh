# Round 2: broker GPU waits sleep-poll instead of spinning (A/B), sandbox GPU tests
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step np600_poll 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
step np600_spin 300 env BEE_BROKER_WAIT=spin python bench.py --steps 600 --materialized-steps 0 --frontends 2
