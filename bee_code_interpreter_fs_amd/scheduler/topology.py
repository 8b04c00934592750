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


def slot_cpus(gpu: Optional[int], sysfs: str = "/sys", allowed: Optional[Set[int]] = None) -> List[int]:
    """CPUs for the slot of HIP device ``gpu``: its NUMA node's CPUs that
    this process may use.  [] = no pinning (unknown topology, one NUMA
    node, or no overlap with the allowed set)."""
    if gpu is None:
        return []
    numa = gpu_numa_nodes(sysfs)
    if gpu >= len(numa) or numa[gpu] < 0 or len({n for n in numa if n >= 0}) < 2:
        return []
    if allowed is None:
        try:
            allowed = set(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            allowed = None
    cpus = numa_cpus(numa[gpu], sysfs)
    if allowed is not None:
        cpus = [c for c in cpus if c in allowed]
    return cpus
