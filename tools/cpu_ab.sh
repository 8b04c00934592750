#!/bin/bash
# Interleaved A/B of service-side CPU knobs on the headline bench (one box):
# each variant is an environment for the whole service (daemons, zygotes,
# sandboxes inherit it); every run appends its JSON line, labelled, to
# gpurun_out/cpu_ab.jsonl.  Variants: "name=VAR=val;VAR=val" ("base" = none;
# values may hold commas; ARGS=--flag+value adds bench.py arguments).
#   bash tools/cpu_ab.sh STEPS ROUNDS base "nosetsid=BEE_SANDBOX_SETSID=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=$1; ROUNDS=$2; shift 2
WARMUP=${WARMUP:-20}  # WARMUP=5 with STEPS=20: the driver's command
OUT=$R/gpurun_out/cpu_ab.jsonl
for round in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}
    vars=""
    [ "$spec" != "$name" ] && vars=${spec#*=}
    envs=()
    IFS=';' read -ra kvs <<< "$vars"
    extra=()
    for kv in "${kvs[@]}"; do
      if [ "${kv%%=*}" = "ARGS" ]; then read -ra extra <<< "${kv#ARGS=}"; extra=("${extra[@]//+/ }");  # ARGS=--frontends+2
      elif [ -n "$kv" ]; then envs+=("$kv"); fi
    done
    echo "[cpu_ab] round $round $name ${envs[*]}" >&2
    line=$(env "${envs[@]}" timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps $STEPS --warmup $WARMUP ${extra[*]} 2>>$R/gpurun_out/cpu_ab.err | grep '^{' | tail -1)
    rc=$?
    if [ $rc -ne 0 ] || [ -z "$line" ]; then echo "[cpu_ab] $name failed rc=$rc" >&2; exit 1; fi
    python3 -c "
import json, sys
d = json.loads(sys.argv[1]); s = d['executors'][0].get('sandbox_cpu', {})
print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'p50': d['p50_latency_ms'],
                  'errors': d['errors'], 'cpu_ms_per_exec': d.get('cpu_ms_per_exec'), 'sandbox_cpu': s,
                  'p50_phase_ms': d.get('p50_phase_ms'), 'node_bound': d.get('node_bound'), 'gpu_time': d.get('gpu_time')}))
" "$line" "$name" "$round" >> $OUT
  done
done
echo "[cpu_ab] done" >&2
