# Round 2 session 3 checkpoint 4 (early huge-page arenas): GPU suite, smoke, default benches
source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python bench.py
step bench_default_2 400 python bench.py
