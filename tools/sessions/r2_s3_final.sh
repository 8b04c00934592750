# Round 2 session 3 final: smoke + two default bench runs (3 front-ends per GPU)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step final_1 400 python bench.py
step final_2 400 python bench.py
