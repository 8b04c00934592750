source tools/gpu_steps.sh
step gputests2 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step nnbench 300 python tools/gemm_nn_bench.py
step b26_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b26_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b26_default 300 python bench.py --gpus 1
