# GEMM lab session: A/B of schedule variants + PMC passes (each its own run)
source tools/gpu_steps.sh
step gemm_lab 400 python tools/gemm_lab.py
export TMPDIR=/tmp
PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
for v in 0 1 -1; do
  step pmc_v$v 120 rocprofv3 --pmc $PMC1 -d gpurun_out/pmc_v$v -o run --output-format csv -- python3 tools/gemm_lab.py --one $v --reps 30
done
