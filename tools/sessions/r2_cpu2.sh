# Round 2: bootstrap env cache + broker client without HELLO; sandbox GPU tests + 3 benches
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step np600_1 300 python bench.py --steps 600 --materialized-steps 0
step np600_2 300 python bench.py --steps 600 --materialized-steps 0
step default 400 python bench.py
