# Round 2: daemon CPU by thread role on the headline payload
source tools/gpu_steps.sh
export TMPDIR=/tmp
step np600_fe2 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
