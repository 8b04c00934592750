"""GPU -> NUMA -> CPU topology of the node, for pinning each GPU slot's
executor daemon (and everything it forks: zygotes, sandboxes, its kernel
broker) and each front-end replica to the CPUs next to its MI355X.

The service is CPU-bound (every Execute forks a sandbox and runs Python);
on a 2-socket 8-GPU node, a slot whose processes wander to the far socket
pays cross-socket memory traffic on every fork and every broker copy.

Sources (no ROCm tools needed): KFD topology nodes (the HIP device order:
GPU nodes in node order, the ones with SIMDs), their PCI location, the PCI
device's ``numa_node``, and the node's ``cpulist``.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional, Set


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def parse_cpulist(text: str) -> List[int]:
    """"0-3,8,10-11" -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in (text or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus: List[int]) -> str:
    cpus = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def gpu_numa_nodes(sysfs: str = "/sys") -> List[int]:
    """NUMA node of each GPU in HIP device order (-1 where unknown)."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        props = _read(os.path.join(base, str(n), "properties")) or ""
        kv: Dict[str, int] = {}
        for line in props.splitlines():
            parts = line.split()
            if len(parts) == 2 and parts[1].lstrip("-").isdigit():
                kv[parts[0]] = int(parts[1])
        if kv.get("simd_count", 0) <= 0:
            continue  # a CPU node
        loc, dom = kv.get("location_id", -1), kv.get("domain", 0)
        numa = -1
        if loc >= 0:
            bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}"
            v = _read(os.path.join(sysfs, "bus", "pci", "devices", bdf, "numa_node"))
            numa = int(v) if v and v.lstrip("-").isdigit() else -1
        out.append(numa)
    return out


def numa_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    return parse_cpulist(_read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) or "")


def cpu_quota(cgroup_fs: str = "/sys/fs/cgroup", proc_cgroup: str = "/proc/self/cgroup") -> float:
    """CPUs' worth of time per period this process's cgroup may use: the
    smallest cgroup v2 ``cpu.max`` quota/period on its path (or the v1
    ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``); 0 = no quota or unknown."""
    best = 0.0

    def take(q: float) -> None:
        nonlocal best
        if q > 0 and (best == 0 or q < best):
            best = q

    own = ""
    for line in (_read(proc_cgroup) or "").splitlines():
        if line.startswith("0::"):
            own = line[3:]
    if own:
        path = own.strip("/")
        parts = path.split("/") if path else []
        for i in range(len(parts), -1, -1):
            v = _read(os.path.join(cgroup_fs, *parts[:i], "cpu.max"))
            if v and v.split()[0] != "max":
                q, per = v.split()[:2]
                take(int(q) / int(per))
    for d in ("cpu", "cpu,cpuacct"):
        q, per = _read(os.path.join(cgroup_fs, d, "cpu.cfs_quota_us")), _read(os.path.join(cgroup_fs, d, "cpu.cfs_period_us"))
        if q and per and q.lstrip("-").isdigit() and int(q) > 0 and int(per) > 0:
            take(int(q) / int(per))
    return best


def core_order(cpus: List[int], sysfs: str = "/sys") -> List[int]:
    """``cpus`` with one logical CPU per physical core first (in CPU order),
    then the cores' SMT siblings."""
    first, rest = [], []
    for c in cpus:
        sib = parse_cpulist(_read(os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology",
                                               "thread_siblings_list")) or str(c))
        (first if not sib or c == min(sib) else rest).append(c)
    return first + rest


def slot_cpus(gpu: Optional[int], sysfs: str = "/sys", allowed: Optional[Set[int]] = None,
              slots: Optional[List[Optional[int]]] = None, quota: Optional[float] = None,
              factor: float = 2.0) -> List[int]:
    """CPUs for the slot of HIP device ``gpu``: its NUMA node's CPUs that
    this process may use (when the GPUs span several NUMA nodes), and --
    when the job's CPU quota (``cpu_quota``) is far below the CPUs it may run
    on -- only ``factor`` x quota of them in all, split between the slots
    (``slots``: every slot's GPU) and physical cores first.  A 16-CPU quota on
    a 256-CPU host otherwise spreads the service over 16 L3 slices and lets
    bursts of runnable threads spend the quota early in a period and stall
    until its end (cpu.stat nr_throttled).  On MI355X, pinned to 32 CPUs:
    4.8-5.2 vs 5.8-7.2 ms of CPU per Execute, throughput within the boxes'
    noise on driver-length runs and lower on 600-step runs
    (profiles/archive/r3_cpu_quota_pinning_ab.log), so the service's default factor
    is 0 (config.cpu_quota_pin_factor).  [] = no pinning."""
    if gpu is None:
        return []
    if allowed is None:
        try:
            allowed = set(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            allowed = None
    numa = gpu_numa_nodes(sysfs)
    by_numa = gpu < len(numa) and numa[gpu] >= 0 and len({n for n in numa if n >= 0}) >= 2
    cpus: List[int] = []
    if by_numa:
        cpus = numa_cpus(numa[gpu], sysfs)
        if allowed is not None:
            cpus = [c for c in cpus if c in allowed]
    q = cpu_quota() if quota is None else quota
    if q > 0 and factor > 0 and allowed:
        budget = max(2, int(factor * q + 0.999))
        if budget < len(allowed):
            slots = [g for g in (slots or [gpu]) if g is not None] or [gpu]
            per = max(2, -(-budget // len(slots)))
            if by_numa:  # the slots of this NUMA node split its CPUs
                peers = [g for g in slots if g < len(numa) and numa[g] == numa[gpu]]
                pool = cpus
            else:
                peers, pool = slots, sorted(allowed)
            k = peers.index(gpu) if gpu in peers else 0
            ordered = core_order(pool, sysfs)
            chunk = ordered[k * per:(k + 1) * per] or ordered[:per]
            return sorted(chunk)
    return cpus if by_numa else []
