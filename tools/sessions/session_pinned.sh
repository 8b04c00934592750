# broker reductions into pinned host slots: GPU suite, served-path profile, bench
source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step prof_served 300 bash tools/prof_served.sh 300
step bench_np600a 300 python bench.py --steps 600
step bench_np600b 300 python bench.py --steps 600
