# scaling rehearsal on one GPU (ranks fold onto the device; the gang check
# needs real GPUs and reports that) + burst vs sustained single-GPU runs
source tools/gpu_steps.sh
step bench_a 300 python bench.py --steps 30
step bench_b 300 python bench.py --steps 30
step bench_long 300 python bench.py --steps 300
step torchrun4 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 30 --warmup 3
