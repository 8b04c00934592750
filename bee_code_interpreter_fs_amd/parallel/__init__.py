"""Multi-GPU support: gang sandboxes and RCCL over xGMI.

The reference has no collectives; multi-GPU user jobs are a
north-star addition.  A request with ``gpus=N`` reserves N whole MI355X
(``LocalGpuPoolBackend._acquire_gang`` + daemon reservations) and the lead
executor launches one rank per GPU with the rendezvous environment built by
:func:`rank_env` — every rank sees the whole gang (``HIP_VISIBLE_DEVICES``
lists all N devices, rank r uses ``cuda:r``) so RCCL can use peer-to-peer
xGMI between them.  Inside the sandbox, :func:`init_process_group` is the
one-liner a user script needs.

:func:`rccl_allreduce_sweep` runs the native ``bee-rccl-bench`` (one process
driving all GPUs) to measure bus bandwidth against the 7 x ~153 GB/s xGMI
budget of an MI355X.
"""

from __future__ import annotations

import json
import os
import subprocess
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
RCCL_BENCH = os.path.join(ROOT, "bee_code_interpreter_fs_amd", "bin", "bee-rccl-bench")

XGMI_LINKS_PER_GPU = 7
XGMI_LINK_GBPS = 153.0  # per direction, per link


def rank_env(rank: int, world: int, gpus: List[int], master_port: int, rdzv: Optional[str] = None) -> Dict[str, str]:
    """Environment of gang rank ``rank`` (mirrors what the executor sets,
    csrc/executor/sandbox.cpp run_job): ``BEE_GANG_RDZV`` is the FileStore in
    the gang's private directory that ``init_process_group()`` uses by
    default (runtime/sandbox_patches.py); RCCL's bootstrap stays on loopback."""
    env = {
        "RANK": str(rank),
        "LOCAL_RANK": str(rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(world),
        "MASTER_ADDR": "127.0.0.1",
        "MASTER_PORT": str(master_port),
        "HIP_VISIBLE_DEVICES": ",".join(str(g) for g in gpus),
        "NCCL_SOCKET_IFNAME": "lo",
    }
    if rdzv:
        env["BEE_GANG_RDZV"] = rdzv
    return env


def init_process_group(backend: Optional[str] = None):
    """Initialise torch.distributed from the gang sandbox environment.

    ``backend`` defaults to "nccl" (RCCL on ROCm) when a GPU is visible, else
    "gloo"; each rank binds ``cuda:LOCAL_RANK``.
    """
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    from ..runtime.sandbox_patches import next_rendezvous

    rdzv = next_rendezvous()  # a fresh FileStore file per init
    if rdzv:
        dist.init_process_group(backend, init_method=rdzv, rank=rank, world_size=world)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world


def busbw_budget_gbps(world: int) -> float:
    """Upper bound of all-reduce bus bandwidth per GPU: the node is fully
    connected (one xGMI link between every pair of its 8 GPUs), so a gang of
    ``world`` GPUs reaches its peers over world - 1 links of ~153 GB/s each
    (all 7 at world = 8), if RCCL spreads its channels over all of them."""
    if world <= 1:
        return float("inf")
    return min(world - 1, XGMI_LINKS_PER_GPU) * XGMI_LINK_GBPS


def rccl_allreduce_sweep(
    gpus: Optional[int] = None, min_bytes: str = "1K", max_bytes: str = "1G", iters: int = 20, timeout: float = 600,
    dtype: str = "f32",
) -> List[dict]:
    """Run ``bee-rccl-bench`` (``dtype`` f32 or bf16) and return its JSON records."""
    cmd = [RCCL_BENCH, "--min", str(min_bytes), "--max", str(max_bytes), "--iters", str(iters), "--dtype", dtype]
    if gpus:
        cmd += ["--gpus", str(gpus)]
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if proc.returncode != 0:
        raise RuntimeError(f"bee-rccl-bench failed ({proc.returncode}): {proc.stderr[-2000:]}")
    return [json.loads(line) for line in proc.stdout.splitlines() if line.startswith("{")]
