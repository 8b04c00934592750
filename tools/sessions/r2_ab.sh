# Round 2: A/B of pooled prefault and huge-page zygote heap on the final build (interleaved, 2 runs each)
source tools/gpu_steps.sh
export TMPDIR=/tmp
for i in 1 2; do
  step base_$i 300 python bench.py --steps 600 --materialized-steps 0
  step noprefault_$i 300 env BEE_PREFAULT=0 python bench.py --steps 600 --materialized-steps 0
  step nothp_$i 300 env BEE_ZYGOTE_THP=0 python bench.py --steps 600 --materialized-steps 0
done
