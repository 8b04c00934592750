source tools/gpu_steps.sh
step gputests45 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke45 300 python -c "import __graft_entry__ as g; g.smoke()"
step b45_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b45_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b45_short3 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b45_600 300 python bench.py --gpus 1
