# A/B: pooled-sandbox prefault on (default) vs off (BEE_PREFAULT=0), interleaved
source tools/gpu_steps.sh
step np_pf1a 300 python bench.py --steps 600
step np_pf0a 300 env BEE_PREFAULT=0 python bench.py --steps 600
step np_pf1b 300 python bench.py --steps 600
step np_pf0b 300 env BEE_PREFAULT=0 python bench.py --steps 600
step he_pf1 300 python bench.py --workload hello --steps 600
step he_pf0 300 env BEE_PREFAULT=0 python bench.py --workload hello --steps 600
