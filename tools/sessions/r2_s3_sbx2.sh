# Round 2 session 3: broker poll default + pooled-phase stamps (redirect/view/paths/ready)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 12
