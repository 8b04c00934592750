# Round 2 session 3: zygote-built stdio layers; pooled-phase stamps, sandbox + example GPU tests, 2 benches
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 12
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step np600_1 300 python bench.py --steps 600 --materialized-steps 0
step np600_2 300 python bench.py --steps 600 --materialized-steps 0
