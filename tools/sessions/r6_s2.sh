#!/bin/bash
# Round 6, session 2: GPU timing per segment (two event reads per wait) --
# its test, and an interleaved A/B against timing off.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/cpu_ab.jsonl
step broker_timing 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_sandbox_gpu.py -k "broker_times or payload_runs"
step timing_ab 1200 bash tools/cpu_ab.sh 600 2 base timingoff=BEE_BROKER_GPU_TIMING=0
