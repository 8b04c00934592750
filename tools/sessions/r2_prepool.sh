# Round 2: request-independent run setup moved into the pooled phase; sandbox tests + headline x2
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step np600_a 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
step np600_b 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
