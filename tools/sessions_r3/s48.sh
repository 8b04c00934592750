source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests48 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke48 300 python -c "import __graft_entry__ as g; g.smoke()"
step b48_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b48_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b48_short3 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b48_600 300 python bench.py --gpus 1
