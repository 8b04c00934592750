# Round 2 session 3: fork cost by zygote preload, torchrun 2-rank rehearsal (ranks fold onto the one GPU), offered-load sweep
source tools/gpu_steps.sh
export TMPDIR=/tmp
step forkprobe 120 bash -c 'for m in "" numpy bee_code_interpreter_fs_amd.ops "numpy,bee_code_interpreter_fs_amd.ops"; do python tools/probe/fork_preload_probe.py "$m"; done'
step torchrun2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 100 --warmup 5 --materialized-steps 0
step conc12 300 python bench.py --steps 300 --concurrency 12 --materialized-steps 0
step conc16 300 python bench.py --steps 300 --concurrency 16 --materialized-steps 0
