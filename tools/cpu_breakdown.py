"""CPU cost per request by process role, while bench.py runs (psutil).

    python tools/cpu_breakdown.py [bench.py args...]

Samples the bench process tree twice during the timed phase and prints cores
used by: bench clients, front-end, executor daemon (incl. kernel broker),
zygotes (forking), and single-use workers (reaped children of zygotes)."""

import collections
import json
import os
import subprocess
import sys
import time

import psutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def role(proc: psutil.Process, bench_pid: int) -> str:
    if proc.pid == bench_pid:
        return "bench_clients"
    cmd = " ".join(proc.cmdline())
    if "bee-executor" in cmd:
        return "executor_daemon"
    if "runtime.zygote" in cmd:
        # zygotes are children of the daemon; pooled workers are forks of zygotes
        parent = proc.parent()
        return "zygote" if parent is not None and "bee-executor" in " ".join(parent.cmdline()) else "worker_live"
    if "bee_code_interpreter_fs_amd" in cmd:
        return "frontend"
    return "other"


def snap(bench_pid: int):
    out = collections.Counter()
    try:
        procs = [psutil.Process(bench_pid)] + psutil.Process(bench_pid).children(recursive=True)
    except psutil.Error:
        return out
    for p in procs:
        try:
            r = role(p, bench_pid)
            t = p.cpu_times()
            out[r] += t.user + t.system
            if r == "zygote":
                out["worker_reaped"] += t.children_user + t.children_system
        except psutil.Error:
            pass
    return out


def main():
    args = sys.argv[1:] or ["--steps", "400", "--warmup", "3"]
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), *args], stdout=subprocess.PIPE, text=True)
    # wait for the service + warmup (the bench prints only at the end)
    time.sleep(float(os.environ.get("CPU_BD_DELAY", "25")))
    a, t0 = snap(p.pid), time.time()
    time.sleep(float(os.environ.get("CPU_BD_WINDOW", "4")))
    b, dt = snap(p.pid), time.time() - t0
    res = p.communicate()[0].strip().splitlines()
    bench = json.loads(res[-1]) if res and res[-1].startswith("{") else {}
    rps = bench.get("value") or 1
    cores = {k: round((b[k] - a[k]) / dt, 2) for k in sorted(set(a) | set(b))}
    print(json.dumps({"rps": rps, "cores": cores, "total_cores": round(sum(cores.values()), 2),
                      "cpu_ms_per_request": {k: round(v / rps * 1e3, 3) for k, v in cores.items()}}))


if __name__ == "__main__":
    main()
