#!/bin/bash
# rocprofv3 counter passes of the f64 / f32 GEMM against torch.matmul (one
# kernel per run, one counter group per pass); tools/gemm_fp_pmc.py tabulates.
#   [IMPLS="bk torch"] [PASSES="1 2"] [TAG=x] bash tools/gemm_fp_pmc.sh DTYPE SIZE
# (kernel env overrides such as BK_GEMM_FP_RS pass through; TAG names them)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
DT=${1:-float32}
N=${2:-4096}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P4="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES TA_BUSY_avr GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
for impl in ${IMPLS:-bk torch}; do
  for pass in ${PASSES:-1 2}; do
    eval C=\$P$pass
    d=pmc_${DT}_${N}_${impl}${TAG:+_$TAG}_$pass
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/$d -o run -- \
      python3 $R/tools/gemm_fp_one.py --impl $impl --dtype $DT --size $N --reps 10 > $R/gpurun_out/$d.log 2>&1
  done
done
echo pmc-done
