# Round 2: event-deferred broker frees + vectorized column sums, re-measured
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_np600 300 python bench.py --steps 600
step prof_served 300 bash tools/prof_served.sh 200
