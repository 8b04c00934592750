# Round 2 session 3: HIP hardware queues for the broker's per-session streams (GPU_MAX_HW_QUEUES 4 default vs 2 vs 1), interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 1 2; do
step q4_$i 300 python bench.py --steps 600 --materialized-steps 0
step q2_$i 300 env GPU_MAX_HW_QUEUES=2 python bench.py --steps 600 --materialized-steps 0
step q1_$i 300 env GPU_MAX_HW_QUEUES=1 python bench.py --steps 600 --materialized-steps 0
done
