source tools/gpu_steps.sh
step kbench 300 python tools/bench_kernels.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_kernels -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/prof_kernels.log 2>&1
echo "[step] rocprof rc=$?"
grep dispatch $GRAFT_REPO_ROOT/gpurun_out/prof_kernels.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm -o pmc -- python3 $GRAFT_REPO_ROOT/tools/gemm_one.py --variant 3 --reps 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm.log 2>&1
echo "[step] pmc rc=$?"
tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm.log
