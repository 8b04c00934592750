# What a headline sandbox has mapped when it exits (its teardown unmaps all
# of it): the payload, then its smaps rollup, page-table size (VmPTE) and
# mapping count, as one JSON line.  Run through the service:
#   python tools/probe/sandbox_debug.py --n 3 --payload tools/probe/teardown_probe_payload.py
import json
import time

import beekern as bk


def gpu_intensive_computation():
    n = 10**8
    a = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    b = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    c = bk.matmul(a, b.T)
    x = bk.random.rand(n)
    result = bk.sum(bk.square(x))
    rows = bk.sum(c, axis=1)
    checksum = bk.sum(rows)
    return result, checksum, a, b, rows


t0 = time.time()
result, checksum, a, b, rows = gpu_intensive_computation()
print("Result:", result, "checksum:", checksum)
roll = {}
for line in open("/proc/self/smaps_rollup"):
    p = line.split()
    if len(p) >= 3 and p[2] == "kB":
        roll[p[0].rstrip(":")] = int(p[1])
status = {}
for line in open("/proc/self/status"):
    k, _, v = line.partition(":")
    if k in ("VmPTE", "VmRSS", "RssAnon", "RssFile", "RssShmem", "Threads"):
        status[k] = v.strip()
kinds = {}
for line in open("/proc/self/maps"):
    p = line.split()
    name = p[5] if len(p) > 5 else ""
    k = "anon" if not name else name if name.startswith("[") else ("file-" + p[1])
    kinds[k] = kinds.get(k, 0) + 1
import sys
sys.stderr.write("TEARDOWN " + json.dumps({"rollup_kb": roll, "status": status, "vmas": kinds}) + "\n")

# the same mappings' fork + exit: a grandchild that exits at once (its CPU is
# the copy-on-fork's child side plus exit's teardown), with / without a
# session of its own
import os
import statistics


def child_cpu(setsid: bool, raw: bool = False) -> list:
    import ctypes

    libc = ctypes.CDLL(None)
    out, flt = [], []
    for _ in range(7):
        pid = libc.fork() if raw else os.fork()  # raw: no interpreter after-fork work
        if pid == 0:
            if setsid:
                libc.setsid()
            libc._exit(0)
        _, _, ru = os.wait4(pid, 0)
        out.append((ru.ru_utime + ru.ru_stime) * 1e3)
        flt.append(ru.ru_minflt)
    return [round(statistics.median(out), 3), statistics.median(flt)]


sys.stderr.write("TEARDOWN_FORK " + json.dumps({"os_fork": child_cpu(False), "os_fork_setsid": child_cpu(True),
                                                "raw_fork": child_cpu(False, True),
                                                "raw_fork_setsid": child_cpu(True, True)}) + "\n")
