"""The multi-GPU request path end to end on CPU, with *virtual* GPU slots.

bench.py's N>1 runs (the driver's 8-GPU pass) send ``Execute(gpus=N)``
through the service: the local pool claims N slots (``_acquire_gang``),
drains them in every daemon (``/v1/reserve`` under the node flock), and the
lead executor starts N ranks with the rendezvous environment.  Slots here are
GPU ids 0 and 1 on a machine without GPUs -- ``HIP_VISIBLE_DEVICES`` is only
an environment variable to the scheduler -- and the ranks all-reduce over
gloo instead of RCCL, so everything but the collective's transport is the
8-GPU code path.
"""

import textwrap

import pytest

from .harness import ServiceHarness, ensure_native_executor

GANG_GLOO = textwrap.dedent(
    """
    import os, torch, torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.tensor([float(rank + 1)])
    dist.all_reduce(x)
    print(f"rank{rank}/{world} sum={x.item()} local={os.environ['LOCAL_RANK']} vis={os.environ.get('HIP_VISIBLE_DEVICES')}")
    dist.destroy_process_group()
    """
)


@pytest.fixture(scope="module")
def two_slot_service(tmp_path_factory):
    ensure_native_executor()
    h = ServiceHarness(
        str(tmp_path_factory.mktemp("gangsvc")),
        gpu_ids=[0, 1],
        broker_enabled=False,
        worker_warm_gpu=False,
        workers_per_gpu_target=1,
        default_timeout=120.0,
    )
    h.start()
    yield h
    h.stop()


def test_gang_request_spans_both_slots(two_slot_service):
    h = two_slot_service
    r = h.call(h.ctx.code_executor.execute(source_code=GANG_GLOO, gpus=2, nprocs=2, timeout=120), timeout=300)
    assert r.exit_code == 0, r.stderr
    lines = sorted(l for l in r.stdout.splitlines() if l.startswith("rank"))
    assert len(lines) == 2, r.stdout
    assert all("sum=3.0" in l and "vis=0,1" in l for l in lines), lines
    assert sorted(r.gpu_ids) == [0, 1]


def test_single_gpu_requests_spread_and_gang_after(two_slot_service):
    """Single-GPU traffic uses both slots; a gang request afterwards still
    gets both (reservations released, nothing left draining)."""
    import asyncio

    h = two_slot_service

    async def burst():
        return await asyncio.gather(*(h.ctx.code_executor.execute(source_code="print(6 * 7)") for _ in range(6)))

    rs = h.call(burst(), timeout=300)
    assert all(r.exit_code == 0 and r.stdout == "42\n" for r in rs)
    assert {g for r in rs for g in r.gpu_ids} == {0, 1}
    r = h.call(h.ctx.code_executor.execute(source_code=GANG_GLOO, gpus=2, nprocs=2, timeout=120), timeout=300)
    assert r.exit_code == 0 and r.stdout.count("sum=3.0") == 2, (r.stdout, r.stderr)


GANG_REINIT = textwrap.dedent(
    """
    import os, torch, torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    for round_ in range(3):  # init -> destroy -> init: a fresh FileStore file each time
        dist.init_process_group("gloo")
        x = torch.tensor([float(rank + 1 + round_)])
        dist.all_reduce(x)
        print(f"round{round_} rank{rank} sum={x.item()}")
        dist.destroy_process_group()
    """
)


def test_gang_reinitialises_process_group(two_slot_service):
    """The default (FileStore) rendezvous survives init / destroy / init in
    one job: each init takes a fresh file (sandbox_patches.next_rendezvous),
    where re-using the first group's file could hang or fail."""
    h = two_slot_service
    r = h.call(h.ctx.code_executor.execute(source_code=GANG_REINIT, gpus=2, nprocs=2, timeout=120), timeout=300)
    assert r.exit_code == 0, r.stderr
    for k in range(3):
        assert r.stdout.count(f"round{k} ") == 2 and f"sum={3.0 + 2 * k}" in r.stdout, r.stdout


def _slot_status(h, i=0):
    return h.call(h.ctx.code_executor.slots[i].executor.get_json("/v1/status"), timeout=30)


def test_gang_ranks_come_from_the_warm_set(two_slot_service):
    """The lead daemon of an aligned block keeps a warm rank set for it
    (config.gang_warm_sizes): a gang request takes it -- no rank is forked
    on the request path -- and a new set is warmed behind it; while none is
    ready, a gang starts cold as before."""
    import time

    h = two_slot_service
    deadline = time.time() + 90
    while _slot_status(h)["gang_warm"].get("0,1") != "ready" and time.time() < deadline:
        time.sleep(0.2)
    st = _slot_status(h)
    assert st["gang_warm"] == {"0,1": "ready"}, st["gang_warm"]
    assert _slot_status(h, 1)["gang_warm"] == {}  # slot 1 leads no aligned block
    hits, cold = st["gang_warm_hits"], st["gang_cold_starts"]
    r = h.call(h.ctx.code_executor.execute(source_code=GANG_GLOO, gpus=2, nprocs=2, timeout=120), timeout=300)
    assert r.exit_code == 0 and r.stdout.count("sum=3.0") == 2, (r.stdout, r.stderr)
    st = _slot_status(h)
    assert st["gang_warm_hits"] == hits + 1 and st["gang_cold_starts"] == cold, st
    assert r.timings_ms["acquire"] < 100.0, r.timings_ms  # no fork + warm-up on the request path
