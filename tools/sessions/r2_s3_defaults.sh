# Round 2 session 3: bench defaults 600 timed / 50 warm-up steps per client; two default runs + torchrun 2-rank rehearsal (ranks fold onto the one GPU)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step def_1 400 python bench.py
step def_2 400 python bench.py
step torchrun2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 100 --warmup 5 --materialized-steps 0
