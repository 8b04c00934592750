# Round 2 session 3: payload per-op breakdown; broker GPU-wait poll schedule A/B (interleaved on one box)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step breakdown 400 python tools/payload_breakdown.py
step base_1 300 python bench.py --steps 600 --materialized-steps 0
step rel8_1 300 env BEE_BROKER_POLL=2,50,8 python bench.py --steps 600 --materialized-steps 0
step rel4_1 300 env BEE_BROKER_POLL=2,50,4 python bench.py --steps 600 --materialized-steps 0
step base_2 300 python bench.py --steps 600 --materialized-steps 0
step rel8_2 300 env BEE_BROKER_POLL=2,50,8 python bench.py --steps 600 --materialized-steps 0
step rel4_2 300 env BEE_BROKER_POLL=2,50,4 python bench.py --steps 600 --materialized-steps 0
