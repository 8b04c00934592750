# Round 2 session 3: HIP hardware queues A/B, round 3 (4 vs 2 vs 1, three interleaved repetitions)
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 3 4 5; do
step q1_$i 300 env GPU_MAX_HW_QUEUES=1 python bench.py --steps 600 --materialized-steps 0
step q4_$i 300 python bench.py --steps 600 --materialized-steps 0
step q2_$i 300 env GPU_MAX_HW_QUEUES=2 python bench.py --steps 600 --materialized-steps 0
done
