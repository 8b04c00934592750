# Round 2 session 3: zygote heap grown from a 2 MB boundary + arenas switched before zygote.py's imports; memory rollups, A/B vs BEE_ZYGOTE_HEAP_ALIGN=0, interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
step sbxdebug 300 python tools/probe/sandbox_debug.py --n 4
for i in 1 2 3; do
step al_$i 300 python bench.py --steps 600 --warmup 50 --materialized-steps 0
step noal_$i 300 env BEE_ZYGOTE_HEAP_ALIGN=0 python bench.py --steps 600 --warmup 50 --materialized-steps 0
done
