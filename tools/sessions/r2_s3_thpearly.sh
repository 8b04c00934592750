# Round 2 session 3: pymalloc arenas on huge pages from interpreter start-up (preloaded shim); sandbox GPU tests, memory rollups, A/B vs BEE_ZYGOTE_THP_EARLY=0 interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sandbox_tests 600 python -u -m pytest tests/test_sandbox_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 4
for i in 1 2 3; do
step early_$i 300 python bench.py --steps 600 --warmup 50 --materialized-steps 0
step late_$i 300 env BEE_ZYGOTE_THP_EARLY=0 python bench.py --steps 600 --warmup 50 --materialized-steps 0
done
