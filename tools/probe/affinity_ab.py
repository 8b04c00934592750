"""Does the job's CFS bandwidth quota throttle the service?  Runs bench.py as
a child process with an optional CPU affinity (inherited by the whole
service tree) and reports the cgroup's cpu.stat throttling counters around
it.

    python tools/probe/affinity_ab.py --cpus 16 -- --gpus 1 --steps 20 --warmup 5
    (--cpus 0: no pinning; N > 0: the first N CPUs of the GPU's NUMA node)
"""

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as fh:
            return {k: int(v) for k, v in (line.split() for line in fh if len(line.split()) == 2)}
    except OSError:
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpus", type=int, default=0)
    ap.add_argument("--smt", action="store_true", help="N CPUs as N/2 cores + their SMT siblings (cpu + ncpu/2)")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = [x for x in a.rest if x != "--"]
    from bee_code_interpreter_fs_amd.scheduler.topology import slot_cpus

    cpus = None
    if a.cpus > 0:
        near = slot_cpus(0) or sorted(os.sched_getaffinity(0))
        if a.smt:
            half = (os.cpu_count() or 2) // 2
            cores = [c for c in near if c < half][: a.cpus // 2]
            cpus = sorted(cores + [c + half for c in cores])
        else:
            cpus = near[: a.cpus]
    s0, t0 = cpu_stat(), time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *rest], cwd=ROOT, capture_output=True, text=True,
                       preexec_fn=(lambda: os.sched_setaffinity(0, cpus)) if cpus else None, timeout=600)
    s1 = cpu_stat()
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    out = json.loads(line[-1]) if line else {"error": p.stderr[-1000:]}
    d = {k: s1.get(k, 0) - s0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")}
    print(json.dumps({"cpus": a.cpus, "smt": a.smt, "cpu_list": cpus and ",".join(map(str, cpus)), "wall_s": round(time.time() - t0, 2),
                      "cpu_stat_delta": d, "value": out.get("value"), "p50_ms": out.get("p50_latency_ms"),
                      "cpu_ms_per_exec": out.get("cpu_ms_per_exec"), "bench": out}), flush=True)
    sys.exit(p.returncode)


if __name__ == "__main__":
    main()
