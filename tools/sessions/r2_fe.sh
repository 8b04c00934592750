# Round 2: front-end replicas / load-generator A/B on the headline payload
source tools/gpu_steps.sh
export TMPDIR=/tmp
step np600_fe1 300 python bench.py --steps 600 --materialized-steps 0 --frontends 1
step np600_fe2 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
step np600_fe3 300 python bench.py --steps 600 --materialized-steps 0 --frontends 3
step np600_c16 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2 --concurrency 16
