source tools/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step bench1 400 python bench.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
