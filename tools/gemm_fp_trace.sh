#!/bin/bash
# Kernel traces of the f64 / f32 GEMM and torch.matmul at the sizes where the
# MFMA kernel trails torch: which library kernel (macro tile, split) torch
# runs, and our kernel's own time apart from its C memset.
#   bash tools/gemm_fp_trace.sh [SIZES...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SIZES=${*:-1024 1536 2048}
for dt in float64 float32; do
  for n in $SIZES; do
    for impl in bk torch; do
      d=$R/gpurun_out/trace_${dt}_${n}_${impl}
      timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $d -o run -- \
        python3 $R/tools/gemm_fp_one.py --impl $impl --dtype $dt --size $n --reps 20 > $d.log 2>&1 || exit $?
    done
  done
done
echo trace-done
