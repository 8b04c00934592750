#!/bin/bash
# Round-5 validation on one box: the GPU suite, smoke, the driver's command
# twice, one 600-step run.
source tools/gpu_steps.sh
step r5v_gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r5v_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r5v_bench_driver1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step r5v_bench_driver2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step r5v_bench_600 300 python bench.py --gpus 1
