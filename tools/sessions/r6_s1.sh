#!/bin/bash
# Round 6, session 1: the tightened GEMM bounds and the broker's GPU timing on
# the box, the driver's bench command, and GPU timing on/off A/B.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gemm_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm or matmul or gemv" 
step broker_timing 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_sandbox_gpu.py -k "broker_times or payload_runs"
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step timing_ab 900 bash tools/cpu_ab.sh 600 1 base timingoff=BEE_BROKER_GPU_TIMING=0
