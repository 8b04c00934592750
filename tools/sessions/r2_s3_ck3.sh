# Round 2 session 3 checkpoint 3 (zygote mallopt, sandbox thresholds restored): GPU suite, smoke, benches
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step np600_1 300 python bench.py --steps 600 --materialized-steps 0
step np600_2 300 python bench.py --steps 600 --materialized-steps 0
