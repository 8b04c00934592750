#!/bin/bash
# Tile-shape / K-group / stagger variants of the f64 / f32 GEMM against
# torch.matmul at the sizes where it trails (env overrides of
# csrc/kernels/gemm_fp.hip's launch choice); one JSON line per size with the
# variant's label, gpurun_out/gemm_fp_sweep.jsonl.
#   bash tools/gemm_fp_sweep.sh "label ENV=V ..." ...
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/gemm_fp_sweep.jsonl
DT=${DTYPES:-float64 float32}
SZ=${SIZES:-1024 1536 2048}
for spec in "$@"; do
  set -- $spec
  label=$1; shift
  echo "[sweep] $label $*"
  timeout -k 10 240 env "$@" python3 tools/gemm_fp_bench.py --sizes $SZ --dtypes $DT --rounds ${ROUNDS:-5} --reps 10 ${EXTRA:-} \
    | python3 -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); d['label']='$label'; print(json.dumps(d), flush=True)" >> $OUT || exit $?
done
echo sweep-done
