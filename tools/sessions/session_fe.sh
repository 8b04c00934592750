# front-end replicas with clients spread evenly over replica ports
source tools/gpu_steps.sh
step fe1a 300 python bench.py --steps 100 --frontends 1
step fe2a 300 python bench.py --steps 100 --frontends 2
step fe1b 300 python bench.py --steps 100 --frontends 1
step fe2b 300 python bench.py --steps 100 --frontends 2
step tr2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 50 --warmup 3
step tr4 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 4 --steps 30 --warmup 3
