# Round 2: GEMM PMC at 4096^3 -- shipped 4-wave TN kernel, the [K][N] kernel, hipBLASLt (one pass each, kernel trace only)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAIT_ANY,SQ_WAVE_CYCLES,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_tn -o run -- python tools/gemm_one.py --variant 5 --size 4096 --reps 20 > gpurun_out/pmc_tn.log 2>&1 && echo tn ok &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_nn -o run -- python tools/gemm_one.py --nn --size 4096 --reps 20 > gpurun_out/pmc_nn.log 2>&1 && echo nn ok &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_blas -o run -- python tools/gemm_one.py --variant 0 --size 4096 --reps 20 > gpurun_out/pmc_blas.log 2>&1 && echo blas ok
