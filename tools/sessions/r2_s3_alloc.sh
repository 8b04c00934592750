# Round 2 session 3: allocator asks the driver outside its lock; full GPU suite, bench, served-path profile
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step np600 300 python bench.py --steps 600 --materialized-steps 0
step prof_served 300 bash tools/prof_served.sh 200
