# Round 2 session 3: HIP hardware queues for the broker's per-session streams (GPU_MAX_HW_QUEUES 4 default vs 8 vs 16), interleaved
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 1 2; do
step q4_$i 300 python bench.py --steps 600 --materialized-steps 0
step q8_$i 300 env GPU_MAX_HW_QUEUES=8 python bench.py --steps 600 --materialized-steps 0
step q16_$i 300 env GPU_MAX_HW_QUEUES=16 python bench.py --steps 600 --materialized-steps 0
done
