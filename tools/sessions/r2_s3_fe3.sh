# Round 2 session 3: front-end replicas per GPU, 2 (default) vs 3 vs 1, interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 1 2 3; do
step fe2_$i 300 python bench.py --materialized-steps 0
step fe3_$i 300 python bench.py --materialized-steps 0 --frontends 3
done
