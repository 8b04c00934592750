#!/bin/bash
# Round 6, session 7: the final tree's wider picture -- every BASELINE config
# the 1-GPU box runs, the 8-slot fold, a served-path kernel + roctx profile,
# and the headline interleaved with the round-5 tree (600 steps x 3).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/bench_suite.jsonl
rm -f gpurun_out/tree_ab.jsonl
step r6_tree_ab 1500 bash tools/tree_ab.sh abtree_r5 600 3
step r6_suite 900 python tools/bench_suite.py
step r6_fold_numpy 400 python bench.py --gpus 8 --fold --steps 100 --warmup 10 --no-gang-check --materialized-steps 0
step r6_served 400 bash tools/prof_served.sh 300
