#!/bin/bash
# rocprofv3 counter passes of the f64 / f32 GEMM against torch.matmul (one
# kernel per run, one counter group per pass); tools/gemm_fp_pmc.py tabulates.
#   bash tools/gemm_fp_pmc.sh DTYPE SIZE
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
DT=${1:-float32}
N=${2:-4096}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for impl in bk torch; do
  for pass in 1 2; do
    eval C=\$P$pass
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/pmc_${DT}_${N}_${impl}_$pass -o run -- \
      python3 $R/tools/gemm_fp_one.py --impl $impl --dtype $DT --size $N --reps 10 > $R/gpurun_out/pmc_${DT}_${N}_${impl}_$pass.log 2>&1
  done
done
echo pmc-done
