# Multi-GPU job inside the sandbox: run with gpus=N; the executor starts N
# ranks with RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT set, one GPU
# each, and RCCL carries the all-reduce over xGMI.  With gpus=1 the script
# forms a world of one.
import os
import socket

import torch
import torch.distributed as dist

if "RANK" not in os.environ:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))

torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
dist.init_process_group("nccl")
rank, world = dist.get_rank(), dist.get_world_size()
t = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(t)
expected = world * (world + 1) / 2
assert float(t[0]) == expected, (float(t[0]), expected)
if rank == 0:
    print(f"allreduce ok world={world} value={float(t[0])}")
dist.destroy_process_group()
