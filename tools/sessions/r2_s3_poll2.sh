# Round 2 session 3: broker GPU-wait poll schedule A/B, round 2 (relative backoff variants, interleaved)
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 1 2; do
step rel8_$i 300 env BEE_BROKER_POLL=2,50,8 python bench.py --steps 600 --materialized-steps 0
step rel12_$i 300 env BEE_BROKER_POLL=2,50,12 python bench.py --steps 600 --materialized-steps 0
step rel8x100_$i 300 env BEE_BROKER_POLL=2,100,8 python bench.py --steps 600 --materialized-steps 0
step rel6_$i 300 env BEE_BROKER_POLL=2,50,6 python bench.py --steps 600 --materialized-steps 0
step rel8m5_$i 300 env BEE_BROKER_POLL=5,50,8 python bench.py --steps 600 --materialized-steps 0
done
