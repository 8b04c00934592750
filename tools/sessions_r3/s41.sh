source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests41 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke41 300 python -c "import __graft_entry__ as g; g.smoke()"
step b41_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b41_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b41_short3 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b41_600 300 python bench.py --gpus 1
step torchrun41 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5
