# Round 2 session 3: zygote glibc allocations kept on the (huge-page collapsed) heap; zygote memory rollups, A/B vs BEE_ZYGOTE_MALLOPT=0, interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 12
for i in 1 2 3; do
step mo_$i 300 python bench.py --steps 600 --materialized-steps 0
step nomo_$i 300 env BEE_ZYGOTE_MALLOPT=0 python bench.py --steps 600 --materialized-steps 0
done
