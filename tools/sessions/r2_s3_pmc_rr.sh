# Round 2 session 3: PMC of the fused Philox->reduce kernel (VALU issue), one counter pass
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_rr -o pmc -- python3 $GRAFT_REPO_ROOT/tools/probe/rand_reduce_bench.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_rr.log 2>&1
echo "[step] pmc rc=$?"
tail -4 $GRAFT_REPO_ROOT/gpurun_out/pmc_rr.log
