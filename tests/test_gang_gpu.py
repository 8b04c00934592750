"""Gang (multi-GPU) Executes through the service on real MI355X GPUs.

A request with ``gpus=N`` reserves N whole GPUs node-wide and runs N ranks
that all-reduce over RCCL/xGMI (BASELINE config 5).  The service here spans
every visible GPU; each gang size N in {2, 4, 8} that fits runs through the
full path -- routing, daemon reservations, rank spawn, the FileStore
rendezvous in the gang's private directory, RCCL -- and is checked for the
sum and for bus bandwidth against the xGMI budget.  (On the one-GPU box the
N > 1 cases skip; the driver's 8-GPU node runs them.)
"""

import tempfile
import textwrap
import time

import pytest

from .harness import ServiceHarness, ensure_native_executor

pytestmark = pytest.mark.gpu

GANG = textwrap.dedent(
    """
    import os, time, torch, torch.distributed as dist
    t0 = time.perf_counter()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    dist.init_process_group("nccl")          # default init: the gang's FileStore
    t_init = time.perf_counter()
    x = torch.full((64 << 20,), float(rank + 1), device="cuda")  # 256 MB f32
    dist.all_reduce(x); torch.cuda.synchronize()
    ok = bool((x[:4096] == world * (world + 1) / 2).all()) and bool((x[-4096:] == world * (world + 1) / 2).all())
    t = time.perf_counter(); iters = 10
    for _ in range(iters):
        dist.all_reduce(x)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / iters
    busbw = 2 * (world - 1) / world * x.numel() * 4 / dt / 1e9
    store = type(dist.distributed_c10d._get_default_store()).__name__
    print(f"rank={rank} ok={ok} busbw_GBps={busbw:.1f} init_ms={(t_init - t0) * 1e3:.0f} store={store}", flush=True)
    dist.destroy_process_group()
    """
)


def _device_count() -> int:
    import torch

    return torch.cuda.device_count()


@pytest.fixture(scope="module")
def node():
    n = _device_count()
    if n < 2:
        pytest.skip(f"gang Executes need >= 2 GPUs (this box has {n})")
    ensure_native_executor()
    h = ServiceHarness(tempfile.mkdtemp(prefix="bee-gang-gpu-"), gpu_ids=list(range(n)), workers_per_gpu_target=1,
                       default_timeout=180.0)
    h.start()
    yield h
    h.stop()


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_gang_allreduce_through_the_service(node, gpus):
    from bee_code_interpreter_fs_amd.parallel import busbw_budget_gbps

    if gpus > _device_count():
        pytest.skip(f"{gpus} GPUs requested, {_device_count()} visible")
    t0 = time.time()
    r = node.call(node.ctx.code_executor.execute(source_code=GANG, gpus=gpus, nprocs=gpus, timeout=180), timeout=400)
    took = time.time() - t0
    assert r.exit_code == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("rank=")]
    assert len(lines) == gpus, r.stdout
    kv = [dict(p.split("=", 1) for p in l.split()) for l in lines]
    assert all(k["ok"] == "True" for k in kv), lines
    assert all(k["store"] == "FileStore" for k in kv), lines  # not a loopback TCPStore
    assert sorted(r.gpu_ids) == list(range(gpus)) or len(set(r.gpu_ids)) == gpus
    busbw = min(float(k["busbw_GBps"]) for k in kv)
    # a real fraction of the 7-link budget, and nothing beyond it
    assert 0.25 * busbw_budget_gbps(gpus) < busbw < 1.05 * busbw_budget_gbps(gpus), (busbw, lines)
    print(f"gang of {gpus}: {took:.2f} s end to end, busbw {busbw:.0f} GB/s, init {max(int(k['init_ms']) for k in kv)} ms")


def test_gangs_and_single_gpu_work_coexist(node):
    """A gang of every GPU while single-GPU requests keep arriving: all
    finish, and the node is idle afterwards (reservations released)."""
    import asyncio

    n = _device_count()
    ex = node.ctx.code_executor

    async def mixed():
        singles = [asyncio.ensure_future(ex.execute(source_code="import beekern as bk; print(float(bk.sum(bk.ones(1000))))"))
                   for _ in range(3 * n)]
        gang = await ex.execute(source_code=GANG, gpus=n, nprocs=n, timeout=180)
        return gang, await asyncio.gather(*singles)

    gang, singles = node.call(mixed(), timeout=600)
    assert gang.exit_code == 0 and gang.stdout.count("ok=True") == n, gang.stderr[-2000:]
    assert all(s.exit_code == 0 and s.stdout == "1000.0\n" for s in singles)
    st = node.call(ex.status())
    assert all(s["inflight"] == 0 and not s["reserved"] for s in st["slots"]), st
