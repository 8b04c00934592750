"""An 8-GPU node rehearsed on CPU: 8 virtual GPU slots (executors pinned to
GPU ids 0..7 that need not exist; gang ranks all-reduce over gloo), with
single-GPU traffic and 8-GPU gangs mixed -- the scheduling the driver's
8-GPU scaling run exercises with RCCL.

* no starvation: gangs interleaved with a stream of 1-GPU requests all
  finish, and the 1-GPU requests keep flowing around them;
* a gang rank that dies releases every slot (fail-fast: its peers, stuck in
  a collective, are killed after the grace period, not at the timeout);
* a reservation left behind by a front-end that died expires by its TTL.
"""

import asyncio
import textwrap
import time

import pytest

from .harness import ServiceHarness, ensure_native_executor

GANG = textwrap.dedent(
    """
    import os, torch, torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.tensor([float(rank + 1)])
    dist.all_reduce(x)
    if rank == 0:
        print(f"sum={x.item()} world={world}")
    dist.destroy_process_group()
    """
)

# rank 3 dies; the others block the way ranks stuck in an RCCL collective
# do (gloo would notice the dead peer by itself, RCCL waits)
GANG_RANK_DIES = textwrap.dedent(
    """
    import os, signal, time
    rank = int(os.environ["RANK"])
    if rank == 3:
        time.sleep(0.5)
        os.kill(os.getpid(), signal.SIGKILL)
    time.sleep(300)
    """
)


@pytest.fixture(scope="module")
def node8(tmp_path_factory):
    ensure_native_executor()
    h = ServiceHarness(
        str(tmp_path_factory.mktemp("node8")),
        gpu_ids=list(range(8)),
        broker_enabled=False,
        worker_warm_gpu=False,
        workers_per_gpu_target=0,
        light_workers_per_gpu_target=1,
        min_workers_per_gpu_target=1,
        min_zygotes_per_gpu=1,
        light_zygotes_per_gpu=1,
        default_timeout=120.0,
        gang_failure_grace_s=3.0,
    )
    h.start()
    yield h
    h.stop()


def _slots_idle(h):
    st = h.call(h.ctx.code_executor.status())
    return all(s["inflight"] == 0 and not s["reserved"] for s in st["slots"]), st


def test_gangs_and_single_gpu_traffic_mix_without_starvation(node8):
    h = node8
    ex = h.ctx.code_executor

    async def mixed():
        singles = [asyncio.ensure_future(ex.execute(source_code="import time; time.sleep(0.2); print('one')", gpus=1))
                   for _ in range(24)]
        gangs = []
        for _ in range(2):
            gangs.append(await ex.execute(source_code=GANG, gpus=8, nprocs=8, timeout=120))
        return gangs, await asyncio.gather(*singles)

    t0 = time.time()
    gangs, singles = h.call(mixed(), timeout=600)
    assert all(g.exit_code == 0 and "sum=36.0 world=8" in g.stdout for g in gangs), [(g.stdout, g.stderr[-300:]) for g in gangs]
    assert sorted(g.gpu_ids for g in gangs) == [list(range(8))] * 2
    assert all(r.exit_code == 0 and r.stdout == "one\n" for r in singles)
    assert len({g for r in singles for g in r.gpu_ids}) >= 4  # 1-GPU work spread over the node
    assert time.time() - t0 < 400
    idle, st = _slots_idle(h)
    assert idle, st


def test_dead_gang_rank_releases_every_slot(node8):
    h = node8
    t0 = time.time()
    r = h.call(h.ctx.code_executor.execute(source_code=GANG_RANK_DIES, gpus=8, nprocs=8, timeout=100), timeout=300)
    took = time.time() - t0
    assert r.exit_code != 0
    assert "Gang aborted" in r.stderr, r.stderr[-500:]
    assert took < 60, took  # fail-fast, not the 100 s timeout
    idle, st = _slots_idle(h)
    assert idle, st
    ok = h.call(h.ctx.code_executor.execute(source_code=GANG, gpus=8, nprocs=8, timeout=120), timeout=300)
    assert ok.exit_code == 0 and "sum=36.0" in ok.stdout, ok.stderr[-500:]


def test_orphaned_reservation_expires(node8):
    """A front-end that reserved a GPU and died never releases it; the
    daemon's TTL does."""
    h = node8
    slot = h.ctx.code_executor.slots[5]
    resp = h.call(slot.executor.post("/v1/reserve", {"ttl": 2.0, "wait": 5.0}))
    assert resp.status_code == 200
    t0 = time.time()
    body = {"source_code": "print('after ttl')", "timeout": 30}
    r = h.call(slot.executor.post("/v1/execute", body, timeout=60), timeout=90)
    assert r.status_code == 200 and r.json()["stdout"] == "after ttl\n"
    assert time.time() - t0 >= 1.5  # held back until the reservation lapsed
