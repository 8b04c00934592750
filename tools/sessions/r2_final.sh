# Round 2 checkpoint: full GPU suite, smoke, default bench, 600-step bench x2, served-path profile
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step np600_a 300 python bench.py --steps 600
step np600_b 300 python bench.py --steps 600 --materialized-steps 0
step prof_served 300 bash tools/prof_served.sh 300
