# perf session: CPU per request by role, 2-rank torchrun rehearsal (device
# folding on one GPU), rocprofv3 kernel stats of the bench
source tools/gpu_steps.sh
step cpu_bd 300 python tools/cpu_breakdown.py --steps 800 --warmup 3
step torchrun2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 3
export TMPDIR=/tmp
step rocprof_bench 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 20 --warmup 3
