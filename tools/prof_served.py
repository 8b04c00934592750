"""rocprofv3 of the SERVED path: one bee-executor daemon (its kernel broker
launches every beekern kernel of minimal/light sandboxes) under the profiler,
driven with Execute requests of the headline payload over its Unix socket.

    tools/prof_served.sh   (wraps the three steps below for a gpurun session)

    python tools/prof_served.py cmd  DIR          # the daemon command line (one arg per line)
    python tools/prof_served.py drive DIR --n 200  # wait for the socket, run the payload N times
    python tools/prof_served.py shutdown DIR      # graceful stop via POST /v1/shutdown
    python tools/prof_served.py stop PID          # SIGTERM the daemon (PID or its child), wait

The daemon runs with BEE_PROFILE_DAEMON_ONLY=1 so its sandboxes do not
inherit the profiler (sandbox processes are forked from zygotes; the kernels
of light/minimal sandboxes run in the daemon anyway)."""

import argparse
import asyncio
import json
import os
import signal
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAYLOAD = os.path.join(ROOT, "examples", "benchmark_numpy_gpu.py")


def sock_path(d: str) -> str:
    return os.path.join(d, "executor.sock")


def cmd(d: str) -> None:
    from bee_code_interpreter_fs_amd.scheduler.executor_process import ExecutorProcess

    ex = ExecutorProcess("prof", os.path.join(d, "sandboxes"), gpus="0", target=1, light_target=2, broker=True,
                         light_zygotes=1, extra_args=["--min-target", "2", "--min-zygotes", "1",
                                                    "--nano-target", "8", "--nano-zygotes", "2"])
    for a in ex.command(sock_path(d)):
        print(a)


async def _drive(d: str, n: int, conc: int) -> dict:
    from bee_code_interpreter_fs_amd.scheduler.uds_http import UdsHttpClient

    path = sock_path(d)
    deadline = time.time() + 120
    while not os.path.exists(path):
        if time.time() > deadline:
            raise SystemExit("daemon socket never appeared")
        await asyncio.sleep(0.2)
    client = UdsHttpClient(path)
    for _ in range(150):  # warm pool (30 s at most)
        st = (await client.request("GET", "/v1/status", None, 10)).json()
        if st.get("ready_nano", 0) >= 1:
            break
        await asyncio.sleep(0.2)
    src = open(PAYLOAD).read()
    collect = os.path.join(d, "objects")
    os.makedirs(collect, exist_ok=True)
    lat, bad = [], 0
    left = [n]

    async def one():
        nonlocal bad
        while left[0] > 0:
            left[0] -= 1
            t = time.perf_counter()
            body = {"source_code": src, "timeout": 120, "collect_dir": collect, "mode": "nano", "files": {}}
            r = await client.request("POST", "/v1/execute", json.dumps(body).encode(), 300)
            lat.append((time.perf_counter() - t) * 1e3)
            if r.status_code != 200 or r.json().get("exit_code") != 0:
                bad += 1

    await asyncio.gather(*(one() for _ in range(conc)))
    return {"requests": n, "errors": bad, "p50_ms": round(statistics.median(lat), 3)}


def shutdown(d: str) -> None:
    """Graceful stop through the daemon's own socket (the profiler owns its
    SIGTERM handler), then wait for the daemon to exit."""
    from bee_code_interpreter_fs_amd.scheduler.uds_http import UdsHttpClient

    async def go():
        return await UdsHttpClient(sock_path(d)).request("POST", "/v1/shutdown", b"{}", 10)

    print(json.dumps({"shutdown": asyncio.run(go()).status_code}), flush=True)


def stop(pid: int) -> None:
    def exe(p):
        try:
            return os.readlink(f"/proc/{p}/exe")
        except OSError:
            return ""

    target = pid
    if not exe(pid).endswith("bee-executor"):
        try:
            kids = open(f"/proc/{pid}/task/{pid}/children").read().split()
        except OSError:
            kids = []
        target = next((int(k) for k in kids if exe(int(k)).endswith("bee-executor")), pid)
    os.kill(target, signal.SIGTERM)
    for _ in range(300):
        if not os.path.exists(f"/proc/{target}"):
            return
        time.sleep(0.1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["cmd", "drive", "shutdown", "stop"])
    ap.add_argument("arg")
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--concurrency", type=int, default=8)
    a = ap.parse_args()
    if a.what == "cmd":
        cmd(a.arg)
    elif a.what == "drive":
        print(json.dumps(asyncio.run(_drive(a.arg, a.n, a.concurrency))), flush=True)
    elif a.what == "shutdown":
        shutdown(a.arg)
    else:
        stop(int(a.arg))


if __name__ == "__main__":
    main()
