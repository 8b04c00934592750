# Multi-GPU job inside the sandbox: run with gpus=N; the executor starts N
# ranks with RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT set, one GPU
# each, and RCCL carries the all-reduce over xGMI.
import os

import torch
import torch.distributed as dist

dist.init_process_group("nccl")
rank, world = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
t = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(t)
expected = world * (world + 1) / 2
assert float(t[0]) == expected, (float(t[0]), expected)
if rank == 0:
    print(f"allreduce ok world={world} value={float(t[0])}")
dist.destroy_process_group()
