# Round 2: finer broker poll steps; headline bench x2
source tools/gpu_steps.sh
export TMPDIR=/tmp
step np600_a 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
step np600_b 300 python bench.py --steps 600 --materialized-steps 0 --frontends 2
