# Round 2 re-entry baseline: GPU suite, smoke, driver-default bench, kernel-trace profile of the bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step bench_np600 300 python bench.py --steps 600
