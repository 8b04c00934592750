#!/bin/bash
# The 8-GPU topology folded onto one GPU (8 daemons / brokers / HIP contexts,
# 64 clients): headline and hello, 100 steps each.
source tools/gpu_steps.sh
step r5_fold_numpy 400 python bench.py --gpus 8 --fold --steps 100 --warmup 10 --no-gang-check --materialized-steps 0
step r5_fold_hello 400 python bench.py --gpus 8 --fold --steps 100 --warmup 10 --no-gang-check --workload hello
