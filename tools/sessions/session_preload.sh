# kernel-module preload in the broker: GPU suite, served-path profile (first-request outliers), bench
source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step prof_served 300 bash tools/prof_served.sh 300
step bench_np600 300 python bench.py --steps 600
