"""Gang sandboxes on CPU: nprocs=2 ranks launched by the native executor with
torch.distributed rendezvous env, all-reducing over gloo (the same path an
8-GPU RCCL job takes, minus the GPUs)."""

import asyncio
import os
import tempfile

import pytest

from bee_code_interpreter_fs_amd.config import Config
from bee_code_interpreter_fs_amd.parallel import rank_env
from bee_code_interpreter_fs_amd.scheduler.executor_process import ExecutorProcess

from .harness import ensure_native_executor

GANG = """
import os, torch, torch.distributed as dist
dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
x = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(x)
print(f"rank{dist.get_rank()} sum={x.item()} world={dist.get_world_size()}")
open(f"rank{dist.get_rank()}.txt", "w").write(str(x.item()))
dist.destroy_process_group()
"""


def test_rank_env():
    env = rank_env(1, 4, [4, 5, 6, 7], 29500)
    assert env["RANK"] == "1" and env["WORLD_SIZE"] == "4" and env["HIP_VISIBLE_DEVICES"] == "4,5,6,7"


def test_gang_of_two_ranks_allreduce(tmp_path):
    ensure_native_executor()

    async def go():
        ex = ExecutorProcess("gang", str(tmp_path / "sb"), gpus="", target=1)
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            resp = await ex.post(
                "/v1/execute",
                {"source_code": GANG, "nprocs": 2, "gpus": "", "timeout": 120, "collect_dir": str(tmp_path)},
                timeout=200,
            )
            return resp.status_code, resp.json()
        finally:
            await ex.close()

    status, body = asyncio.run(go())
    assert status == 200, body
    assert body["exit_code"] == 0, body["stderr"]
    lines = sorted(body["stdout"].split())
    assert "rank0" in body["stdout"] and "rank1" in body["stdout"]
    assert "sum=3.0" in body["stdout"]
    # both ranks share one workspace: both files come back
    assert set(body["files"]) == {"/workspace/rank0.txt", "/workspace/rank1.txt"}


def test_gang_reservation_blocks_and_releases(tmp_path):
    ensure_native_executor()

    async def go():
        ex = ExecutorProcess("resv", str(tmp_path / "sb"), gpus="", target=1)
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            r = await ex.post("/v1/reserve", {"ttl": 30, "wait": 5})
            assert r.status_code == 200 and r.json()["drained"]
            # a normal job waits while the reservation holds ...
            job = asyncio.ensure_future(ex.post("/v1/execute", {"source_code": "print(7)"}, timeout=60))
            await asyncio.sleep(0.5)
            assert not job.done()
            # ... a gang job bypasses it ...
            g = await ex.post("/v1/execute", {"source_code": "print(8)", "gang": True}, timeout=60)
            assert g.json()["stdout"] == "8\n"
            # ... and release lets the queued job through
            await ex.post("/v1/release", {})
            done = await asyncio.wait_for(job, 30)
            return done.json()
        finally:
            await ex.close()

    out = asyncio.run(go())
    assert out["stdout"] == "7\n"


def test_idle_sandboxes_are_recycled(tmp_path):
    """--max-idle: warm sandboxes older than the bound are replaced."""
    ensure_native_executor()

    async def go():
        ex = ExecutorProcess("idle", str(tmp_path / "sb"), gpus="", target=1, extra_args=["--max-idle", "1"])
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            await asyncio.sleep(3.0)
            metrics = (await ex.client.request("GET", "/metrics", None, 10)).text
            r = await ex.post("/v1/execute", {"source_code": "print(5)"}, timeout=60)
            return metrics, r.json()
        finally:
            await ex.close()

    metrics, body = asyncio.run(go())
    recycled = [l for l in metrics.splitlines() if l.startswith("bee_executor_idle_recycled_total")]
    assert recycled and float(recycled[0].split()[-1]) >= 1, metrics
    assert body["stdout"] == "5\n"


def test_gang_ranks_get_the_operator_rccl_env(tmp_path):
    """--gang-env (config gang_rccl_env): every gang rank gets the operator's
    RCCL policy, a request's own NCCL_* entry wins over it, and a non-gang
    sandbox gets none of it."""
    ensure_native_executor()
    code = "import os\nprint(os.environ.get('RANK'), os.environ.get('NCCL_IB_DISABLE'), os.environ.get('NCCL_PROTO'))\n"

    async def go():
        ex = ExecutorProcess("gang", str(tmp_path / "sb"), gpus="", target=1,
                             extra_args=["--gang-env", "NCCL_IB_DISABLE=1,NCCL_PROTO=Simple"])
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            gang = await ex.post("/v1/execute", {"source_code": code, "nprocs": 2, "gpus": "", "timeout": 60,
                                                 "env": {"NCCL_PROTO": "LL128"}, "collect_dir": str(tmp_path)},
                                 timeout=120)
            one = await ex.post("/v1/execute", {"source_code": code, "timeout": 60, "collect_dir": str(tmp_path)},
                                timeout=120)
            return gang.json(), one.json()
        finally:
            await ex.close()

    gang, one = asyncio.run(go())
    assert gang["exit_code"] == 0, gang["stderr"]
    assert sorted(gang["stdout"].splitlines()) == ["0 1 LL128", "1 1 LL128"], gang["stdout"]
    assert one["stdout"] == "None None None\n", one


def test_cpu_only_pools_take_the_cpu_targets(tmp_path):
    """Without a broker the nano_cpu / min_cpu kinds fold into nano / min
    (stdlib scripts run in the nano pool), so those pools are sized for the
    CPU-only targets too rather than for the GPU-script ones -- and a zygote
    of the kind starts even when only the *_cpu target is set."""
    ensure_native_executor()

    async def go(extra):
        ex = ExecutorProcess("cpuonly", str(tmp_path / f"sb{len(extra)}"), gpus="", target=1,
                             light_target=1, light_zygotes=1,
                             extra_args=["--min-zygotes", "1", "--nano-zygotes", "1", *extra])
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            for _ in range(600):
                st = await ex.get_json("/v1/status")
                if st["ready_nano"] >= st["nano_target"] and st["ready_min"] >= st["min_target"]:
                    break
                await asyncio.sleep(0.1)
            r = await ex.post("/v1/execute", {"source_code": "print(6)", "mode": "nano_cpu"}, timeout=60)
            return st, r.json()
        finally:
            await ex.close()

    st, body = asyncio.run(go(["--nano-target", "1", "--nano-cpu-target", "3", "--min-target", "1",
                               "--min-cpu-target", "2"]))
    assert st["nano_cpu_target"] == 0 and st["min_cpu_target"] == 0, st  # no broker: no *_cpu pools
    assert st["nano_target"] == 3 and st["min_target"] == 2, st
    assert st["ready_nano"] == 3 and st["ready_min"] == 2, st
    assert body["stdout"] == "6\n"
    st, body = asyncio.run(go(["--nano-target", "0", "--nano-cpu-target", "2", "--min-target", "0"]))
    assert st["nano_target"] == 2 and st["ready_nano"] == 2 and st["min_target"] == 0, st
    assert body["stdout"] == "6\n"


def _metric(text: str, name: str) -> float:
    return float(next(l for l in text.splitlines() if l.startswith((name + " ", name + "{"))).split()[-1])


def test_a_warm_gang_set_that_cannot_start_is_given_up(tmp_path):
    """Fault injection into the warm gang ranks (every one dies in its
    warm-up): the daemon re-spawns the set a bounded number of times, then
    reports it "disabled" (its gangs start cold; the service's start-up wait
    accepts that) and stops forking torch ranks for it."""
    ensure_native_executor()

    async def go():
        ex = ExecutorProcess("gangfail", str(tmp_path / "sb"), gpus="", target=1,
                             extra_args=["--gang-warm", "0,1", "--gang-env", "BEE_FAULT_DIE_WARM=1"])
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            states = []
            for _ in range(600):
                st = await ex.get_json("/v1/status")
                states.append(st["gang_warm"].get("0,1"))
                if states[-1] == "disabled":
                    break
                await asyncio.sleep(0.1)
            m0 = _metric((await ex.client.request("GET", "/metrics", None, 10)).text,
                         "bee_executor_worker_spawn_failures_total")
            await asyncio.sleep(2.0)
            m1 = _metric((await ex.client.request("GET", "/metrics", None, 10)).text,
                         "bee_executor_worker_spawn_failures_total")
            r = await ex.post("/v1/execute", {"source_code": "print(4)"}, timeout=60)
            return states, m0, m1, r.json()
        finally:
            await ex.close()

    states, m0, m1, body = asyncio.run(go())
    assert states[-1] == "disabled", states[-10:]
    assert "ready" not in states
    assert m0 >= 3 and m1 == m0, (m0, m1)  # no more ranks forked once given up
    assert body["stdout"] == "4\n"  # the rest of the pool is unaffected


def test_pooled_spawn_faults_are_absorbed(tmp_path):
    """--fault-spawn-fail-rate (config.fault_spawn_fail_rate): a share of
    pooled sandboxes dies in warm-up; the pool refills around them and
    requests are served."""
    ensure_native_executor()

    async def go():
        ex = ExecutorProcess("faults", str(tmp_path / "sb"), gpus="", target=2,
                             extra_args=["--fault-spawn-fail-rate", "0.5"])
        await ex.start()
        try:
            await ex.wait_ready(1, 120)
            outs = []
            for i in range(8):
                r = await ex.post("/v1/execute", {"source_code": f"print({i})"}, timeout=60)
                outs.append(r.json()["stdout"])
            m = _metric((await ex.client.request("GET", "/metrics", None, 10)).text,
                        "bee_executor_worker_spawn_failures_total")
            return outs, m
        finally:
            await ex.close()

    outs, failures = asyncio.run(go())
    assert outs == [f"{i}\n" for i in range(8)]
    assert failures >= 1  # p(no failure in >= 10 spawns at 0.5) < 0.1%
