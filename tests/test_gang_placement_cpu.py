"""Gang ranks placed next to their own GPU, and warm gang sets in admission
(VERDICT r4 "next" #4), on CPU with virtual GPU slots.

* every rank of a gang -- warm (taken from the lead daemon's warm set) or
  cold -- runs on the CPUs of the slot whose GPU it drives
  (``scheduler/topology.slot_cpus``), not on the lead daemon's, although the
  lead daemon's zygote forks them all;
* the idle warm ranks each slot's GPU carries are charged against its HBM
  and host-memory admission up front (``--standing-hbm`` / ``--standing-mem``,
  ``csrc/executor/admission.cpp``): a job that would only fit by ignoring
  them is refused;
* a request whose environment sets a torch init-time variable
  (``PYTORCH_*ALLOC_CONF``) starts its ranks cold -- a warm rank initialised
  torch's allocator before the request existed and would ignore it.

The slots are pinned by ``cpu_quota_override`` x ``cpu_quota_pin_factor``:
2 CPUs each on this 8-CPU runner.
"""

import os
import textwrap
import time

import pytest

from .harness import ServiceHarness, ensure_native_executor

AFFINITY = textwrap.dedent(
    """
    import os
    print("rank", os.environ["RANK"], "cpus", ",".join(map(str, sorted(os.sched_getaffinity(0)))),
          "alloc", os.environ.get("PYTORCH_HIP_ALLOC_CONF", "-"))
    """
)

RANK_HBM = 1 << 30
RANK_MEM = 1 << 30


@pytest.fixture(scope="module")
def four_slots(tmp_path_factory):
    if len(os.sched_getaffinity(0)) < 8:
        pytest.skip("needs 8 CPUs to pin 4 slots to 2 CPUs each")
    ensure_native_executor()
    h = ServiceHarness(
        str(tmp_path_factory.mktemp("gangplace")),
        gpu_ids=[0, 1, 2, 3],
        broker_enabled=False,
        worker_warm_gpu=False,
        workers_per_gpu_target=0,
        light_workers_per_gpu_target=1,
        min_workers_per_gpu_target=0,
        nano_workers_per_gpu_target=1,
        default_timeout=120.0,
        gang_warm_sizes=[2, 4],
        cpu_quota_override=1.0,
        cpu_quota_pin_factor=4.0,
        gang_warm_rank_hbm_bytes=RANK_HBM,
        gang_warm_rank_memory_bytes=RANK_MEM,
    )
    h.start()
    yield h
    h.stop()


def _status(h, i):
    return h.call(h.ctx.code_executor.slots[i].executor.get_json("/v1/status"), timeout=30)


def _ranks(stdout):
    out = {}
    for line in stdout.splitlines():
        parts = line.split()
        if parts and parts[0] == "rank":
            out[int(parts[1])] = ([int(c) for c in parts[3].split(",")], parts[5])
    return out


def _wait_warm(h, key, timeout=120):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if _status(h, 0)["gang_warm"].get(key) == "ready":
            return True
        time.sleep(0.2)
    return False


def test_each_rank_runs_on_its_own_gpus_slot_cpus(four_slots):
    h = four_slots
    backend = h.ctx.code_executor
    want = {g: backend._slot_cpus(g) for g in range(4)}
    assert all(len(c) == 2 for c in want.values()) and len({tuple(c) for c in want.values()}) == 4, want
    assert _wait_warm(h, "0,1,2,3")
    st = _status(h, 0)
    hits, cold = st["gang_warm_hits"], st["gang_cold_starts"]
    warm = h.call(backend.execute(source_code=AFFINITY, gpus=4, nprocs=4, timeout=120), timeout=300)
    assert warm.exit_code == 0, warm.stderr
    st = _status(h, 0)
    assert st["gang_warm_hits"] == hits + 1 and st["gang_cold_starts"] == cold, st
    got = _ranks(warm.stdout)
    assert {r: c for r, (c, _) in got.items()} == {r: want[r] for r in range(4)}, (got, want)
    # a cold gang (its init-time allocator setting forces one): the same placement
    cold_r = h.call(backend.execute(source_code=AFFINITY, gpus=4, nprocs=4, timeout=120,
                                    env={"PYTORCH_HIP_ALLOC_CONF": "expandable_segments:True"}), timeout=300)
    assert cold_r.exit_code == 0, cold_r.stderr
    assert _status(h, 0)["gang_cold_starts"] == cold + 1
    got = _ranks(cold_r.stdout)
    assert {r: c for r, (c, _) in got.items()} == {r: want[r] for r in range(4)}, (got, want)
    assert all(a == "expandable_segments:True" for _, a in got.values()), got
    # a 1-GPU sandbox keeps its own slot's CPUs
    one = h.call(backend.execute(source_code="import os; print(sorted(os.sched_getaffinity(0)))", gpus=1), timeout=120)
    assert one.exit_code == 0 and eval(one.stdout) == want[one.gpu_ids[0]], (one.stdout, one.gpu_ids)


def test_warm_gang_ranks_are_charged_to_admission(four_slots):
    h = four_slots
    backend = h.ctx.code_executor
    # sizes 2 and 4: every slot carries one rank of a pair set and one of the quad set
    for i in range(4):
        adm = _status(h, i)["admission"]
        assert adm["standing_hbm"] == 2 * RANK_HBM, (i, adm)
        assert adm["standing_mem"] == (2 * RANK_MEM if adm["mem_capacity"] > 0 else 0), (i, adm)
    slot = backend.slots[1]
    cap = _status(h, 1)["admission"]["hbm_capacity"]
    assert cap > 2 * RANK_HBM
    # fits the GPU, not what the idle warm ranks leave of it: refused at once
    r = h.call(slot.executor.post("/v1/execute", {"source_code": "print(1)", "hbm_quota": cap - RANK_HBM}), timeout=60)
    assert r.status_code == 400 and "warm gang ranks" in r.json()["detail"], r.text
    ok = h.call(slot.executor.post("/v1/execute", {"source_code": "print(1)", "hbm_quota": cap - 2 * RANK_HBM}),
                timeout=60)
    assert ok.status_code == 200 and ok.json()["stdout"] == "1\n", ok.text
