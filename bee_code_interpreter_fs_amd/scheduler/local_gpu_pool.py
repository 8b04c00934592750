"""LocalGpuPoolBackend: GPU-pinned executor pools on one MI355X node.

Replaces the reference's Kubernetes pod pool (`kubernetes_code_executor.py:
163-279`) for a single 8-GPU node:

* one native ``bee-executor`` per GPU slot, each keeping
  ``workers_per_gpu_target`` warm single-use sandboxes whose HIP context is
  already created on that GPU (HIP_VISIBLE_DEVICES pin);
* admission is the executor daemon's (csrc/executor/sandbox.cpp run_job):
  each GPU's daemon admits at most ``max_inflight_per_gpu`` jobs whose HBM
  quotas (default (288 GB - reserve) / max in-flight) fit its usable HBM,
  and queues the rest in arrival order -- one bound per GPU for every
  front-end replica of the node, where the reference spawns a pod
  synchronously per request when its deque is empty (`:268-272`);
* dispatch routes to the least-loaded healthy GPU as every replica sees it:
  the daemons publish their admitted / waiting jobs, committed HBM and gang
  reservations in a shared load table (scheduler/load_table.py);
* requests that can never fit fail at once: ``hbm_bytes`` above a GPU's
  usable HBM or ``gpus`` above the node's GPU count are INVALID_ARGUMENT;
* multi-GPU requests reserve a gang of whole GPUs atomically: the claimed
  slots stop admitting new work, drain, and the leader's executor launches
  one rank per GPU with torch.distributed rendezvous env (RCCL over xGMI);
* input objects are copied into the sandbox by the executor straight from
  the object store directory and changed files are hard-linked back — no
  bytes go through Python or HTTP;
* a failed slot (executor crash) is marked unhealthy, restarted in the
  background, and the request is retried elsewhere (RuntimeError, 3 tries,
  the reference's retry policy).
"""

from __future__ import annotations

import asyncio
import collections
import functools
import json
import logging
import os
import re
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..config import Config
from ..services.storage import Storage
from .backend import CodeExecutor, ExecuteRequest, ExecutionResult
from .executor_process import ExecutorProcess
from .load_table import LoadTable, open_table
from .topology import format_cpulist, slot_cpus
from .uds_http import UdsHttpError

logger = logging.getLogger("local_gpu_pool")

# JSON list of {index, gpu, address}: set for front-end replica processes
ATTACH_ENV = "BEE_FRONTEND_ATTACH"


def detect_gpus() -> List[int]:
    """Visible MI355X devices without initialising HIP in this process."""
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip().isdigit()]
    try:
        import torch

        n = torch.cuda.device_count()  # does not initialise HIP on this image
        return list(range(n))
    except Exception:
        return []


@dataclass
class Slot:
    index: int
    gpu: Optional[int]  # None = CPU-only slot
    executor: ExecutorProcess
    inflight: int = 0  # this replica's requests on the slot (its daemon bounds all replicas')
    hbm_committed: int = 0
    load: Optional[LoadTable] = None  # the daemon's published load (all replicas)
    healthy: bool = True
    reserved: bool = False  # claimed by a waiting gang: admit nothing new
    executions: int = 0
    failures: int = 0
    last_error: str = ""


@dataclass
class PoolStats:
    executions: int = 0
    failures: int = 0
    queue_wait_ms_sum: float = 0.0
    latency_ms: List[float] = field(default_factory=list)


_QUANTITY = {"": 1, "k": 1000, "M": 1000**2, "G": 1000**3, "T": 1000**4, "P": 1000**5,
             "Ki": 1024, "Mi": 1024**2, "Gi": 1024**3, "Ti": 1024**4, "Pi": 1024**5}


def parse_quantity(v) -> float:
    """A Kubernetes resource quantity ("16Gi", "500m", "2", 1.5) as a number."""
    if isinstance(v, (int, float)):
        return float(v)
    text = str(v).strip()
    if text.endswith("m") and text[:-1].replace(".", "", 1).isdigit():
        return float(text[:-1]) / 1000.0
    for suffix in sorted(_QUANTITY, key=len, reverse=True):
        if suffix and text.endswith(suffix):
            return float(text[: -len(suffix)]) * _QUANTITY[suffix]
    return float(text)


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as fh:
            text = fh.read().strip()
        return int(text) if text.isdigit() else None
    except OSError:
        return None


def host_memory_budget(c: Config) -> int:
    """Host memory the node's sandboxes may commit in all (bytes, 0 = no
    bound): config.host_memory_budget_bytes, or 85% of the smaller of
    MemTotal and this service's cgroup memory limit (v2 memory.max, v1
    memory.limit_in_bytes)."""
    if c.host_memory_budget_bytes < 0:
        return 0
    if c.host_memory_budget_bytes > 0:
        return int(c.host_memory_budget_bytes)
    total = 0
    try:
        with open("/proc/meminfo") as fh:
            for line in fh:
                if line.startswith("MemTotal:"):
                    total = int(line.split()[1]) * 1024
                    break
    except OSError:
        pass
    for path in ("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory/memory.limit_in_bytes"):
        lim = _read_int(path)
        if lim and (total == 0 or lim < total):
            total = lim
    return int(total * 0.85)


def containment_limits(c: Config, slots: int = 1, standing_mem: int = 0) -> dict:
    """Per-sandbox bounds of the whole process tree (csrc/executor/procmon.hpp):
    the reference's ``executor_container_resources`` limits (`config.py:67-68`,
    applied to each pod's container at `kubernetes_code_executor.py:246`)
    mapped onto the local backend -- ``limits.memory`` and ``limits.cpu`` --
    with the APP_SANDBOX_* settings as defaults; plus each of ``slots``
    daemons' share of the host-memory budget (``mem_capacity``), which the
    daemons admit the trees' bounds against (a node of 8 GPUs x 16 admitted
    sandboxes x a 64 GiB bound would otherwise commit 8 TiB).  An automatic
    tree bound is that share, less what the slot's idle warm gang ranks hold
    (``standing_mem``, charged by the daemon up front), over the slot's
    admissible sandboxes."""
    limits = (c.executor_container_resources or {}).get("limits") or {}
    budget = host_memory_budget(c)
    per_slot = budget // max(slots, 1) if budget > 0 else 0
    # what jobs can commit on the slot once its warm gang ranks are charged
    room = max(per_slot - max(int(standing_mem), 0), 0) if per_slot > 0 else 0
    if "memory" in limits:
        mem = int(parse_quantity(limits["memory"]))
    elif c.sandbox_tree_memory_bytes > 0:
        mem = int(c.sandbox_tree_memory_bytes)
    elif room > 0:
        mem = min(max(room // max(c.max_inflight_per_gpu, 1), 2 << 30), 64 << 30)
    else:
        mem = 64 << 30
    if room > 0:
        mem = min(mem, room)  # one sandbox must always be admissible
    cpus = parse_quantity(limits["cpu"]) if "cpu" in limits else float(c.sandbox_cpus)
    return {"memory": max(mem, 0), "tasks": max(int(c.sandbox_max_processes), 0), "cpus": max(cpus, 0.0),
            "mem_capacity": per_slot}


def _listen_ports(c: Config) -> List[int]:
    out = []
    for addr in (c.grpc_listen_addr, c.http_listen_addr):
        try:
            out.append(int(addr.rpartition(":")[2]))
        except ValueError:
            pass
    return out


def isolation_args(c: Config, slot: int, protect: List[str]) -> List[str]:
    """bee-executor flags of the sandbox jail (runtime/jail.py) for slot
    ``slot``: each slot owns a disjoint block of sandbox UIDs."""
    mode = (c.sandbox_isolation or "auto").lower()
    if mode == "off":
        return []
    from ..runtime import jail

    if not jail.available():
        if mode == "on":
            raise RuntimeError("APP_SANDBOX_ISOLATION=on but the native jail (_jail) is not built")
        logger.warning("sandbox isolation: native jail not built; sandboxes run unconfined")
        return []
    args = ["--jail", "1", "--nproc", str(c.sandbox_max_processes), "--mem-limit", str(c.sandbox_memory_bytes)]
    if c.sandbox_uid_base > 0:
        args += ["--uid-base", str(c.sandbox_uid_base + slot * c.sandbox_uid_count),
                 "--uid-count", str(c.sandbox_uid_count)]
    for p in protect:
        args += ["--protect", os.path.abspath(p)]
    return args


SOCKET_HOLDER_TIMEOUT_S = 2.0  # one daemon's answer to the peer guard's socket lookup


class LocalGpuPoolBackend(CodeExecutor):
    def __init__(self, config: Config, storage: Storage, gpu_ids: Optional[List[int]] = None) -> None:
        self.config = config
        self.storage = storage
        ids = detect_gpus() if gpu_ids is None and config.gpu_ids is None else (gpu_ids if gpu_ids is not None else config.gpu_ids)
        self.gpu_ids: List[int] = list(ids or [])
        self.default_gpus = 1 if self.gpu_ids else 0
        self.slots: List[Slot] = []
        self.attached = False
        self._rr = int(os.environ.get("BEE_FRONTEND_INDEX", "0"))
        self._cond: Optional[asyncio.Condition] = None
        self._tasks: set = set()
        self.stats_ = PoolStats()
        self.hbm_capacity = max(config.hbm_total_bytes - config.hbm_reserve_bytes, 0)  # per GPU (--hbm-capacity)
        self._derive_quota()
        # TCP ports sandboxes may not reach: the service's listeners (the
        # entry point adds replica ports it picks before the executors start)
        self.deny_ports: List[int] = sorted({p for p in [*_listen_ports(config), *config.sandbox_deny_ports] if p})

    def _derive_quota(self) -> None:
        """Idle warm gang ranks hold HBM on every GPU their aligned blocks
        cover, charged by each daemon up front (--standing-hbm): the room jobs
        have is what they leave, and the default quota must fit it
        max_inflight times over (it was derived from the whole
        capacity, so with max_inflight=1 every default request was refused)."""
        c = self.config
        self.standing_hbm = (max((self._warm_ranks_on(i) for i in range(len(self.gpu_ids))), default=0)
                             * int(c.gang_warm_rank_hbm_bytes)) if self.gpu_ids else 0
        self.hbm_room = max(self.hbm_capacity - self.standing_hbm, 0)
        self.default_quota = c.hbm_quota_bytes or (self.hbm_room // max(c.max_inflight_per_gpu, 1))

    # ---- lifecycle --------------------------------------------------------------------
    async def start(self) -> None:
        self._cond = asyncio.Condition()
        attach = os.environ.get(ATTACH_ENV)
        if attach:
            # front-end replica: the executors belong to the supervisor process
            for entry in json.loads(attach):
                ex = self._make_executor(entry["index"], entry["gpu"])
                ex.attach(entry["address"])
                self.slots.append(Slot(index=entry["index"], gpu=entry["gpu"], executor=ex,
                                       load=open_table(entry.get("load_table"))))
            self.gpu_ids = [s.gpu for s in self.slots if s.gpu is not None]
            self.default_gpus = 1 if self.gpu_ids else 0
            self._derive_quota()
            self.attached = True
            return
        devices: List[Optional[int]] = list(self.gpu_ids) or [None]
        for i, gpu in enumerate(devices):
            ex = self._make_executor(i, gpu)
            self.slots.append(Slot(index=i, gpu=gpu, executor=ex))
        await asyncio.gather(*(s.executor.start() for s in self.slots))
        await asyncio.gather(*(self._open_load(s) for s in self.slots))
        logger.info("local pool: %d slot(s) on GPUs %s", len(self.slots), self.gpu_ids or "[cpu]")

    async def _open_load(self, slot: Slot) -> None:
        try:
            st = await slot.executor.get_json("/v1/status")
            slot.load = open_table((st.get("admission") or {}).get("load_table"))
        except Exception:  # noqa: BLE001 - routing falls back to this replica's own counts
            slot.load = None

    def attach_spec(self) -> str:
        """What front-end replicas need to share this pool's executors."""
        return json.dumps([{"index": s.index, "gpu": s.gpu, "address": s.executor.address,
                            "load_table": s.load.path if s.load else None} for s in self.slots])

    def _make_executor(self, i: int, gpu: Optional[int]) -> ExecutorProcess:
        c = self.config
        lim = containment_limits(c, slots=max(len(self.gpu_ids), 1),
                                 standing_mem=self._warm_ranks_on(i) * int(c.gang_warm_rank_memory_bytes))
        return ExecutorProcess(
            name=f"slot{i}" + (f"-gpu{gpu}" if gpu is not None else "-cpu"),
            sandbox_root=os.path.join(c.sandbox_root, f"slot{i}"),
            gpus="" if gpu is None else str(gpu),
            target=c.workers_per_gpu_target,
            binary=c.executor_binary,
            python=c.worker_python,
            warm_gpu=c.worker_warm_gpu,
            recursive_scan=c.changed_files_recursive,
            default_timeout=c.default_timeout,
            hbm_quota=self.default_quota if gpu is not None else 0,
            max_output=c.max_output_bytes,
            extra_env={"BEE_WHEELHOUSE": c.wheelhouse} if c.wheelhouse else None,
            light_target=c.light_workers_per_gpu_target,
            broker=c.broker_enabled,
            light_zygotes=c.light_zygotes_per_gpu,
            cpus=self._slot_cpus(gpu) or None,
            extra_args=["--max-idle", str(c.worker_max_idle_s), "--min-target", str(c.min_workers_per_gpu_target),
                        "--min-zygotes", str(c.min_zygotes_per_gpu),
                        "--min-cpu-target", str(c.min_cpu_workers_per_gpu_target),
                        "--nano-target", str(c.nano_workers_per_gpu_target),
                        "--nano-zygotes", str(c.nano_zygotes_per_gpu),
                        "--nano-cpu-target", str(c.nano_cpu_workers_per_gpu_target),
                        "--gang-grace", str(c.gang_failure_grace_s),
                        "--fault-spawn-fail-rate", repr(float(c.fault_spawn_fail_rate or 0.0)),
                        "--gang-warm", ";".join(self._gang_keys_led_by(i)),
                        # gang ranks run next to their own GPU, not the lead's
                        "--gang-cpus", ";".join(f"{g}={format_cpulist(cs)}" for g, cs in
                                                ((g, self._slot_cpus(g)) for g in self.gpu_ids) if cs),
                        # idle warm gang ranks on this GPU, charged up front
                        "--standing-hbm", str(self._warm_ranks_on(i) * c.gang_warm_rank_hbm_bytes if gpu is not None else 0),
                        "--standing-mem", str(self._warm_ranks_on(i) * c.gang_warm_rank_memory_bytes),
                        "--standing-rank-hbm", str(c.gang_warm_rank_hbm_bytes if gpu is not None and self._warm_ranks_on(i) else 0),
                        "--standing-rank-mem", str(c.gang_warm_rank_memory_bytes if self._warm_ranks_on(i) else 0),
                        "--gang-env", ",".join(f"{k}={v}" for k, v in sorted((c.gang_rccl_env or {}).items())
                                               if "," not in f"{k}={v}"),
                        # admission for every front-end replica of the node
                        "--max-inflight", str(max(c.max_inflight_per_gpu, 0)),
                        "--hbm-capacity", str(self.hbm_capacity if gpu is not None else 0),
                        # the reference pod's container limits, per sandbox tree
                        "--sandbox-memory", str(lim["memory"]), "--sandbox-tasks", str(lim["tasks"]),
                        "--mem-capacity", str(lim["mem_capacity"]),
                        "--sandbox-network", c.sandbox_network or "open",
                        "--listen-guard", "1" if c.sandbox_listen_guard else "0",
                        "--sandbox-cpus", repr(lim["cpus"]), "--monitor-ms", str(c.sandbox_monitor_ms),
                        "--deny-ports", ",".join(str(p) for p in self.deny_ports) if c.sandbox_net_layer else "",
                        "--cgroup", c.sandbox_cgroup or "auto", "--cgroup-root", c.sandbox_cgroup_root or "",
                        *isolation_args(c, i, [self.storage.storage_path])],
        )

    def _slot_cpus(self, gpu: Optional[int]) -> List[int]:
        """The CPUs GPU ``gpu``'s slot is pinned to ([] = not pinned)."""
        c = self.config
        if gpu is None or (c.numa_affinity or "auto").lower() == "off":
            return []
        return slot_cpus(gpu, slots=list(self.gpu_ids), factor=c.cpu_quota_pin_factor,
                         quota=c.cpu_quota_override or None)

    def _warm_ranks_on(self, slot: int) -> int:
        """Idle warm gang ranks placed on slot ``slot``'s GPU: one per warm
        gang size whose aligned block covers it (rank r of a set holds the
        block's r-th GPU)."""
        if not self.gpu_ids:
            return 0
        sizes = {int(x) for x in (self.config.gang_warm_sizes or []) if 1 < int(x) <= len(self.gpu_ids)}
        return sum(1 for n in sizes for block in self._aligned_blocks(n) if slot in block)

    def _aligned_blocks(self, n: int) -> List[List[int]]:
        """Slot-index blocks a gang of ``n`` is placed on first: aligned runs
        of n slots (all 8; 0-3 / 4-7; the pairs), each over n distinct GPUs."""
        ids = list(self.gpu_ids)
        out = []
        for i in range(0, len(ids) - n + 1, n):
            block = list(range(i, i + n))
            if len({ids[j] for j in block}) == n:
                out.append(block)
        return out

    def _gang_keys_led_by(self, slot: int) -> List[str]:
        """The warm gang sets slot ``slot``'s daemon keeps: the aligned blocks
        it leads (their first slot), as the GPU list a gang request names."""
        if not self.gpu_ids or slot >= len(self.gpu_ids):
            return []
        keys = []
        for n in sorted({int(x) for x in (self.config.gang_warm_sizes or []) if 1 < int(x) <= len(self.gpu_ids)}):
            for block in self._aligned_blocks(n):
                if block[0] == slot:
                    keys.append(",".join(str(self.gpu_ids[j]) for j in block))
        return keys

    async def wait_ready(self, timeout: float = 300.0) -> None:
        await asyncio.gather(*(s.executor.wait_ready(min(1, self.config.workers_per_gpu_target), timeout) for s in self.slots))

    async def wait_warm(self, timeout: float = 300.0) -> bool:
        """Until every slot's pools are at target (direct, light, minimal
        sandboxes), its zygotes are all up and its broker holds its session
        contexts and reserved memory: what the service reaches before it says
        READY, so its first requests are served like its thousandth (a fresh
        node used to serve its first few hundred 20-35% slower)."""
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout

        def full(st: dict) -> bool:
            return (st.get("zygotes_alive", 0) >= st.get("zygotes", 0)
                    and st.get("ready_direct", 0) >= st.get("target", 0)
                    and st.get("ready_light", 0) >= st.get("light_target", 0)
                    and st.get("ready_min", 0) >= st.get("min_target", 0)
                    and st.get("ready_min_cpu", 0) >= st.get("min_cpu_target", 0)
                    and st.get("ready_nano", 0) >= st.get("nano_target", 0)
                    and st.get("ready_nano_cpu", 0) >= st.get("nano_cpu_target", 0)
                    # warm gang rank sets (their HIP + torch init is seconds of
                    # CPU per rank: done before READY, not inside the first
                    # requests' window)
                    # ("disabled": the set failed to start 3 times; its gangs start cold)
                    and all(v in ("ready", "disabled") for v in (st.get("gang_warm") or {}).values()))

        while loop.time() < deadline:
            try:
                sts = await asyncio.gather(*(s.executor.get_json("/v1/status") for s in self.slots))
                if all(full(st) for st in sts):
                    return True
            except Exception:  # noqa: BLE001 - a daemon still starting
                pass
            await asyncio.sleep(0.1)
        logger.warning("pools not at target after %.0f s; serving anyway", timeout)
        return False

    async def close(self) -> None:
        for t in list(self._tasks):
            t.cancel()
        await asyncio.gather(*(s.executor.close() for s in self.slots), return_exceptions=True)

    def healthy(self) -> bool:
        return any(s.healthy and s.executor.alive() for s in self.slots)

    # ---- routing (admission itself is the daemons') -----------------------------------
    async def socket_holder(self, inode: int) -> Optional[str]:
        """The running sandbox (any slot's) that holds local socket ``inode``,
        or None: the peer guard's question when sandboxes share the service's
        UID (services/peer_guard.py, csrc/executor/sandbox_peers.cpp).

        Each slot is asked with a short time limit of its own (one
        hung daemon stalled every new local connection).  A slot that does
        not answer fails the lookup -- the guard then refuses, fail closed --
        only while its daemon process is alive, i.e. may still run sandboxes;
        a dead daemon's sandboxes died with it (--die-with-parent, procmon),
        so it cannot hold the socket and is skipped."""

        async def ask(slot: Slot):
            try:
                return await asyncio.wait_for(slot.executor.get_json(f"/v1/socket-holder/{int(inode)}"),
                                              SOCKET_HOLDER_TIMEOUT_S)
            except Exception as e:  # noqa: BLE001 - decided per slot below
                if not slot.executor.alive():
                    return {}
                raise RuntimeError(f"slot {slot.index} did not answer the socket-holder lookup "
                                   f"({e.__class__.__name__})") from e

        replies = await asyncio.gather(*(ask(s) for s in self.slots), return_exceptions=True)
        failed = None
        for r in replies:
            if isinstance(r, BaseException):
                failed = failed or r
            elif r.get("sandbox"):
                return str(r.get("worker") or "?")
        if failed is not None:
            raise failed  # a live slot could not say: the guard refuses
        return None

    def _routable(self, slot: Slot) -> bool:
        return slot.healthy and not slot.reserved

    def _load_key(self, slot: Slot, hbm: int):
        """Least-loaded order: the daemon's node-wide view (admitted + waiting
        jobs of every replica, gang reservation, HBM headroom) plus this
        replica's own requests on the slot (those still in transit are not in
        the table yet: a burst would otherwise all pick the same GPU); among
        equally loaded GPUs the one that has admitted the fewest jobs (GPUs
        stay evenly used under uniform load); ties rotate so replicas and
        bursts spread over the GPUs."""
        n = len(self.slots)
        rot = (slot.index - self._rr) % n
        ld = slot.load.read() if slot.load is not None else None
        if ld is None:
            return (0, slot.inflight, slot.hbm_committed, rot)
        no_room = ld.hbm_capacity > 0 and ld.hbm_committed + hbm > ld.hbm_capacity
        return (int(ld.reserved) + int(no_room), ld.depth + slot.inflight, ld.executions, rot)

    async def _acquire_one(self, hbm: int) -> Slot:
        assert self._cond is not None
        async with self._cond:
            while True:
                cands = [s for s in self.slots if self._routable(s)]
                if cands:
                    self._rr += 1
                    slot = min(cands, key=lambda s: self._load_key(s, hbm))
                    slot.inflight += 1
                    slot.hbm_committed += hbm
                    return slot
                if not any(s.healthy for s in self.slots):
                    raise RuntimeError("no healthy executor slot")
                await self._cond.wait()

    async def _acquire_gang(self, n: int, hbm: int) -> List[Slot]:
        assert self._cond is not None
        async with self._cond:
            # claim the n healthy, unreserved slots with the least work, then drain them
            while True:
                free = [s for s in self.slots if s.healthy and not s.reserved]
                if len(free) >= n:
                    break
                await self._cond.wait()
            # an aligned block first (its lead daemon keeps a warm rank set
            # for it, config.gang_warm_sizes), the least busy one; any n
            # healthy slots otherwise
            free_ix = {s.index for s in free}
            blocks = [b for b in self._aligned_blocks(n) if all(i in free_ix for i in b)]
            if blocks:
                by_ix = {s.index: s for s in free}
                best = min(blocks, key=lambda b: (sum(by_ix[i].inflight for i in b), b[0]))
                gang = [by_ix[i] for i in best]
            else:
                gang = sorted(free, key=lambda s: (s.inflight, s.index))[:n]
            for s in gang:
                s.reserved = True
            try:
                while any(s.inflight > 0 for s in gang):
                    await self._cond.wait()
            except BaseException:
                for s in gang:
                    s.reserved = False
                self._cond.notify_all()
                raise
            for s in gang:
                s.inflight += 1
                s.hbm_committed += hbm
            return sorted(gang, key=lambda s: s.index)

    async def _release(self, slots: List[Slot], hbm: int, gang: bool = False) -> None:
        assert self._cond is not None
        async with self._cond:
            for s in slots:
                s.inflight -= 1
                s.hbm_committed -= hbm
                if gang:
                    s.reserved = False
            self._cond.notify_all()

    # ---- execution ------------------------------------------------------------------
    async def run(self, request: ExecuteRequest) -> ExecutionResult:
        last: Optional[BaseException] = None
        for attempt in range(3):
            try:
                return await self._run_once(request)
            except _SlotFailure as e:
                last = e
                logger.warning("executor slot failed (%s); retry %d/2", e, attempt + 1)
                await asyncio.sleep(0.05 * (attempt + 1))
        raise RuntimeError(f"execution failed on every attempt: {last}")

    async def _run_once(self, request: ExecuteRequest) -> ExecutionResult:
        t0 = time.perf_counter()
        hbm = int(request.hbm_bytes) if request.hbm_bytes else self.default_quota
        want = int(request.gpus)
        gang = want > 1
        if want == 0 or not self.gpu_ids:
            hbm = 0
        # requests no GPU of this node can ever take: refused now (they would
        # otherwise wait forever for room that never comes)
        if want > max(len(self.gpu_ids), 1):
            raise ValueError(f"requested {want} GPUs but this node has {len(self.gpu_ids)}")
        # the room idle warm gang ranks leave (a gang's rank runs as one of
        # them, so it may use that rank's share too: csrc/executor/admission.cpp)
        room = self.hbm_room + (int(self.config.gang_warm_rank_hbm_bytes) if gang and self.standing_hbm else 0)
        if hbm > min(room, self.hbm_capacity):
            raise ValueError(f"hbm_bytes {hbm} exceeds the usable HBM of one GPU ({min(room, self.hbm_capacity)} bytes"
                             + (f" after {self.standing_hbm} held by warm gang ranks" if self.standing_hbm else "") + ")")
        slots = await self._acquire_gang(want, hbm) if gang else [await self._acquire_one(hbm)]
        lead = slots[0]
        gang_lock = None
        if gang:
            try:
                gang_lock = await self._reserve_gpus(slots, float(request.timeout or self.config.default_timeout))
            except BaseException:
                await self._release(slots, hbm, gang)
                raise
        t_acq = time.perf_counter()
        try:
            body = {
                "files": {p: self.storage.path_of(h) for p, h in request.files.items()},
                "timeout": float(request.timeout or self.config.default_timeout),
                "collect_dir": self.storage.storage_path,
                "hbm_quota": hbm,
            }
            for p, h in request.files.items():
                if not os.path.isfile(body["files"][p]):
                    raise FileNotFoundError(f"File not found: {h}")
            if request.source_file is not None:
                body["source_file"] = request.source_file
            else:
                body["source_code"] = request.source_code
                code = precompiled_if_repeated(request.source_code)
                if code is not None:
                    body["code"] = code
            offload = self.config.numpy_offload if request.numpy_offload is None else request.numpy_offload
            offload = bool(offload) and want > 0
            if not gang:
                # CPU-only slots too: their executors keep minimal (numpy-only,
                # fast-forking) and light zygotes as well
                body["mode"] = sandbox_mode(request, self.storage)
                if offload and body["mode"] == "min_cpu":
                    # numpy code that will reach the GPU: a sandbox whose broker
                    # session opened while it was pooled
                    body["mode"] = "min"
            if gang:
                body["gpus"] = ",".join(str(s.gpu) for s in slots)
                body["nprocs"] = int(request.nprocs)
                body["gang"] = True
            elif want == 0 and lead.gpu is not None:
                body["gpus"] = ""  # CPU-only sandbox on a GPU slot
            if request.env:
                body["env"] = dict(request.env)
            if offload:
                body["numpy_offload"] = True  # a job field: the pooled sandbox applies it (ops/numpy_offload.py)
            if request.trusted_warm:
                body["cow_trusted"] = True  # the service's own self-warm job (zygote_loop.cpp "Trust")
            try:
                resp = await lead.executor.post("/v1/execute", body, timeout=body["timeout"] + 180.0)
            except (UdsHttpError, OSError, AssertionError) as e:
                self._mark_failed(lead, str(e))
                raise _SlotFailure(f"slot {lead.index}: {e}") from e
            if resp.status_code == 503:
                raise _SlotFailure(f"slot {lead.index}: {resp.text}")
            if resp.status_code != 200:
                detail = _detail(resp)
                raise ValueError(detail) if resp.status_code in (400, 422) else RuntimeError(detail)
            data = resp.json()
        finally:
            if gang:
                await self._unreserve_gpus(slots, gang_lock)
            await self._release(slots, hbm, gang)
        t1 = time.perf_counter()
        timings = dict(data.get("timings_ms") or {})
        timings["queue"] = (t_acq - t0) * 1e3
        timings["service_total"] = (t1 - t0) * 1e3
        lead.executions += 1
        self.stats_.executions += 1
        self.stats_.queue_wait_ms_sum += timings["queue"]
        if data.get("exit_code", 0) != 0:
            self.stats_.failures += 1
        return ExecutionResult(
            stdout=data.get("stdout", ""),
            stderr=data.get("stderr", ""),
            exit_code=int(data.get("exit_code", -1)),
            files=dict(data.get("files") or {}),
            timings_ms=timings,
            gpu_ids=[s.gpu for s in slots if s.gpu is not None] if want else [],
        )

    # ---- cross-process gang reservation ---------------------------------------------
    def _gang_lock_path(self) -> str:
        os.makedirs(self.config.sandbox_root, exist_ok=True)
        return os.path.join(self.config.sandbox_root, "gang.lock")

    async def _reserve_gpus(self, slots: List[Slot], timeout: float) -> int:
        """Front-end replicas share executors, so a gang also reserves its
        GPUs in the daemons: a node-wide flock serialises gangs (no two can
        deadlock holding half each other's GPUs), each daemon stops admitting
        new jobs and drains, the reservation expiring on its own if this
        process dies."""
        import fcntl

        loop = asyncio.get_running_loop()
        fd = os.open(self._gang_lock_path(), os.O_RDWR | os.O_CREAT, 0o600)
        try:
            await loop.run_in_executor(None, fcntl.flock, fd, fcntl.LOCK_EX)
            ttl = timeout + 120.0
            resps = await asyncio.gather(
                *(s.executor.post("/v1/reserve", {"ttl": ttl, "wait": ttl}, timeout=ttl + 30) for s in slots)
            )
            if any(r.status_code != 200 for r in resps):
                raise RuntimeError("could not drain the gang's GPUs: " + ", ".join(r.text for r in resps))
        except BaseException:
            await self._unreserve_gpus(slots, fd)
            raise
        return fd

    async def _unreserve_gpus(self, slots: List[Slot], fd: Optional[int]) -> None:
        await asyncio.gather(*(s.executor.post("/v1/release", {}, timeout=30) for s in slots), return_exceptions=True)
        if fd is not None:
            os.close(fd)  # drops the flock

    def _mark_failed(self, slot: Slot, error: str) -> None:
        slot.failures += 1
        slot.last_error = error
        if not slot.executor.alive():
            slot.healthy = False
            task = asyncio.ensure_future(self._restart(slot))
            self._tasks.add(task)
            task.add_done_callback(self._tasks.discard)

    async def _restart(self, slot: Slot) -> None:
        logger.warning("restarting executor for slot %d (gpu %s)", slot.index, slot.gpu)
        try:
            await slot.executor.close()
            slot.executor = self._make_executor(slot.index, slot.gpu)
            await slot.executor.start()
            slot.healthy = True
        except Exception:
            logger.exception("executor restart failed for slot %d", slot.index)
        finally:
            assert self._cond is not None
            async with self._cond:
                self._cond.notify_all()

    async def status(self) -> dict:
        out = []
        for s in self.slots:
            entry = {
                "slot": s.index,
                "gpu": s.gpu,
                "healthy": s.healthy,
                "inflight": s.inflight,
                "reserved": s.reserved,
                "hbm_committed": s.hbm_committed,
                "executions": s.executions,
            }
            try:
                entry["executor"] = await s.executor.get_json("/v1/status")
            except Exception as e:  # noqa: BLE001
                entry["executor_error"] = str(e)
            out.append(entry)
        return {"backend": "local", "default_hbm_quota": self.default_quota, "slots": out}

    def stats(self) -> dict:
        return {
            "executions": self.stats_.executions,
            "failures": self.stats_.failures,
            "slots": len(self.slots),
            "inflight": sum(s.inflight for s in self.slots),
            "healthy_slots": sum(1 for s in self.slots if s.healthy),
        }


class _SlotFailure(RuntimeError):
    pass


# Libraries that bring their own HIP runtime usage: such scripts get a
# "direct" sandbox whose HIP context is already warm; everything else runs in a
# "light" sandbox whose beekern calls go through the executor's kernel broker.
DIRECT_GPU_MODULES = frozenset(
    {"torch", "torchvision", "torchaudio", "cupy", "jax", "jaxlib", "tensorflow", "triton", "numba", "pycuda", "hip"}
)


def sandbox_mode(request: ExecuteRequest, storage: Storage) -> str:
    source = request.source_code
    if source is None and request.source_file is not None:
        try:
            with open(storage.path_of(request.files[request.source_file]), "rb") as fh:
                source = fh.read(4 << 20).decode("utf-8", errors="replace")
        except (OSError, KeyError, ValueError):
            return "direct"
    return _mode_of_source(source or "")


@functools.lru_cache(maxsize=512)
def _mode_of_source(source: str) -> str:
    """The routing decision is a pure function of the source: re-submitted
    scripts (agents re-running cells, benchmark loops) skip the parse."""
    from ..runtime.deps import imported_modules

    mods = imported_modules(source)
    if DIRECT_GPU_MODULES.intersection(mods):
        return "direct"
    if _DYNAMIC_IMPORT.search(source) or "importlib" in mods or "runpy" in mods:
        # imports the static scan cannot see (importlib, __import__, exec /
        # eval of code strings): a site-enabled sandbox with the science stack,
        # never a `python -S` nano one whose .pth start-up hooks did not run
        return "light"
    if all(m in GPU_API_MODULES or m in _STDLIB for m in mods):
        # beekern + stdlib: a sandbox from a zygote that never imported numpy
        # (executor kind nano; the daemon falls back to a minimal one);
        # stdlib only: the same, with its broker session opened on first use
        return "nano" if GPU_API_MODULES.intersection(mods) else "nano_cpu"
    if all(m in MIN_MODULES or m in _STDLIB for m in mods):
        # numpy/beekern/stdlib only: the fast-forking minimal zygote; scripts
        # that never import beekern take a sandbox whose broker session opens
        # only if used (executor kind min_cpu)
        return "min" if GPU_API_MODULES.intersection(mods) else "min_cpu"
    return "light"


# the builtins only, bare or through the builtins module (builtins.exec(,
# __builtins__.eval(): a method of the same name on anything else
# (re.compile, obj.eval, its `def eval(`) is no dynamic import (ADVICE r4:
# "\bcompile(" sent every re.compile script to the slower light kind);
# importlib / runpy are caught by the module scan
_DYNAMIC_IMPORT = re.compile(r"(?<![\w.])(?:(?:builtins|__builtins__)\s*\.\s*)?(?<!def )"
                             r"(?:__import__|exec|eval|compile)\s*\(|(?<![\w])import_module\s*\(|"
                             r"(?<![\w.])__builtins__\s*\[")

# what the minimal zygote preloads (plus the standard library, imported on
# demand at stdlib speed)
MIN_MODULES = frozenset({"numpy", "beekern", "bee_code_interpreter_fs_amd"})
GPU_API_MODULES = frozenset({"beekern", "bee_code_interpreter_fs_amd"})
_STDLIB = frozenset(getattr(sys, "stdlib_module_names", ()))


@functools.lru_cache(maxsize=256)
def precompiled(source: str) -> Optional[str]:
    """The payload compiled here, once per distinct source, for the sandbox
    to load instead of compiling it on the request path
    (runtime/worker.py load_precompiled; ~0.15-0.3 ms of a sandbox's CPU and
    latency for a 40-line script): base64 of the interpreter's bytecode magic,
    a flag byte ("X": xonsh-lowered, needs the shell runtime; "P": plain) and
    the marshalled code object, compiled exactly as the worker would
    (dont_inherit, optimize 0; file name fixed up by the worker).  None when
    the source does not compile: the sandbox then compiles it itself and
    reports the SyntaxError as `python script.py` would."""
    if len(source) > (256 << 10):
        return None
    import base64
    import importlib.util
    import marshal
    import warnings

    from ..runtime import xsh

    try:
        # a compile that warns (SyntaxWarning for `x is 1`, invalid escapes,
        # ...) is left to the sandbox, so its stderr carries the warning as
        # it did on the first run -- not this replica's stderr
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            lowered = xsh.lower_payload(source)
            code = compile(lowered or source, PRECOMPILED_FILENAME, "exec", dont_inherit=True, optimize=0)
        if caught:
            return None
    except (SyntaxError, ValueError, RecursionError, MemoryError, OverflowError):
        return None
    flag = b"X" if lowered is not None else b"P"
    return base64.b64encode(importlib.util.MAGIC_NUMBER + flag + marshal.dumps(code)).decode("ascii")


PRECOMPILED_FILENAME = "<bee-precompiled>"
_PRECOMPILE = os.environ.get("BEE_PRECOMPILE", "1") != "0"  # A/B switch
_SEEN: "collections.OrderedDict[str, None]" = collections.OrderedDict()
_SEEN_MAX, _SEEN_MAX_LEN = 256, 64 << 10


def precompiled_if_repeated(source: str) -> Optional[str]:
    """precompiled() for a source this replica has seen before (benchmark
    loops, agents re-running a cell): compiling every one-off script here
    would only move the sandbox's compile onto the replica's event loop."""
    if not _PRECOMPILE or len(source) > _SEEN_MAX_LEN:
        return None
    if source in _SEEN:
        _SEEN.move_to_end(source)
        return precompiled(source)
    _SEEN[source] = None
    if len(_SEEN) > _SEEN_MAX:
        _SEEN.popitem(last=False)
    return None


def _detail(resp) -> str:
    try:
        return str(resp.json().get("detail", resp.text))
    except Exception:
        return resp.text
