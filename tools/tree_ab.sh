#!/bin/bash
# Interleaved A/B of two trees' headline on one box: this tree vs another
# checkout built in-tree under the repo (e.g. `git worktree add abtree_r5
# <commit>` + its own build()).  Appends labelled JSON lines to
# gpurun_out/tree_ab.jsonl.   bash tools/tree_ab.sh DIR STEPS ROUNDS [WARMUP]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OTHER=$1; STEPS=$2; ROUNDS=$3; WARMUP=${4:-20}
OUT=$R/gpurun_out/tree_ab.jsonl
for round in $(seq 1 "$ROUNDS"); do
  for tree in this other; do
    dir=$R; [ "$tree" = other ] && dir=$R/$OTHER
    echo "[tree_ab] round $round $tree" >&2
    line=$(cd "$dir" && timeout -k 10 300 python3 bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" 2>>"$R/gpurun_out/tree_ab.err" | grep '^{' | tail -1)
    rc=$?
    if [ $rc -ne 0 ] || [ -z "$line" ]; then echo "[tree_ab] $tree failed rc=$rc" >&2; exit 1; fi
    python3 -c "
import json, sys
d = json.loads(sys.argv[1])
print(json.dumps({'tree': sys.argv[2], 'round': int(sys.argv[3]), 'steps': int(sys.argv[4]), 'value': d['value'],
                  'p50': d['p50_latency_ms'], 'p50_in_sandbox': d.get('p50_in_sandbox_exec_ms'), 'errors': d['errors'],
                  'cpu_ms_per_exec': d.get('cpu_ms_per_exec'), 'node_bound': d.get('node_bound'),
                  'gpu_time': d.get('gpu_time'), 'materialized': (d.get('materialized') or {}).get('value'),
                  'sandbox_cpu': d['executors'][0].get('sandbox_cpu')}))
" "$line" "$tree" "$round" "$STEPS" >> "$OUT"
  done
done
echo "[tree_ab] done" >&2
