#!/bin/bash
# One GPU session: kernel tests, kernel microbench, GEMM A/B, rocprofv3 stats
# of the microbench.  Each step under its own limit; stop on a fault.
source tools/gpu_steps.sh
step ktests 300 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider
step kbench 300 python tools/bench_kernels.py
step gemm_ab 300 python tools/gemm_ab.py --repeats 5
cd /tmp && export TMPDIR=/tmp
step_rocprof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_kernels -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/prof_kernels.log 2>&1
  echo "[step] rocprof rc=$?"
}
step_rocprof
