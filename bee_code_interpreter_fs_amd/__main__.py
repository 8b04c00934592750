"""``python -m bee_code_interpreter_fs_amd``: gRPC + HTTP servers.

Parity with `src/code_interpreter/__main__.py:22-36` (uvicorn + grpc.aio under
one event loop, graceful shutdown); the executor backend (GPU-pinned sandbox
pools) is started before either server accepts requests.

Scale-out (``APP_FRONTEND_PROCESSES`` > 1, local backend): this process
becomes a supervisor that owns the per-GPU native executors and starts N
front-end replicas.  Replicas bind the same gRPC/HTTP ports with
SO_REUSEPORT (the kernel spreads connections), attach to the shared
executors, and coordinate gangs through the daemons' reservation API — a
single Python front-end tops out at a few thousand RPC/s, 8 MI355X pools
serve more.
"""

from __future__ import annotations

import asyncio
import gc
import json
import logging
import os
import secrets
import signal
import socket
import subprocess
import sys
import time
from typing import List

import uvicorn

from .application_context import ApplicationContext
from .config import Config
from .services.grpc_servicer import SELF_WARM_HEADER

logger = logging.getLogger("bee_service")


def _split_addr(addr: str):
    host, _, port = addr.rpartition(":")
    return host or "0.0.0.0", int(port)


def _reuseport_socket(host: str, port: int) -> socket.socket:
    family = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(family, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.setblocking(False)
    return s


def _free_port(host: str) -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


async def _serve(ctx: ApplicationContext, stop: asyncio.Event) -> None:
    host, port = _split_addr(ctx.config.http_listen_addr)
    http = uvicorn.Server(uvicorn.Config(ctx.http_server, host=host, port=port, loop="asyncio", log_level="warning"))
    http.install_signal_handlers = lambda: None  # handled by the caller
    sock = _reuseport_socket(host, port)
    ctx.grpc_server.bind(ctx.config.grpc_listen_addr)
    private = ""
    if os.environ.get("BEE_FRONTEND_INDEX") is not None:
        # a replica also listens on a port of its own, so a client (or an L4
        # balancer) can spread connections evenly instead of by SO_REUSEPORT's
        # 4-tuple hash, which leaves some replicas with several times the
        # connections of others
        ghost, _ = _split_addr(ctx.config.grpc_listen_addr)
        own = os.environ.get("BEE_REPLICA_GRPC_PORT", "0")
        try:
            port = ctx.grpc_server.bind(f"{ghost}:{own}")
        except Exception:  # noqa: BLE001 - taken since the supervisor picked it
            port = 0
        if not port:
            port = ctx.grpc_server.bind(f"{ghost}:0")
        private = f" replica_grpc={ghost}:{port}"
    await ctx.grpc_server.start()
    http_task = asyncio.create_task(http.serve(sockets=[sock]))
    # the start-up heap (modules, descriptors, app objects) out of every later
    # collection's scan: a full collection of a replica then walks only what
    # requests left behind, not ~40 MB of long-lived objects mid-request
    if os.environ.get("BEE_GC_FREEZE", "1") != "0":
        gc.collect()
        gc.freeze()
    print(f"BEE_SERVICE_READY grpc={ctx.config.grpc_listen_addr} http={ctx.config.http_listen_addr}{private}", flush=True)
    try:
        await stop.wait()
    finally:
        http.should_exit = True
        await ctx.grpc_server.stop(grace=5)
        await http_task


def _install_stop(loop) -> asyncio.Event:
    stop = asyncio.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, stop.set)
    return stop


async def main() -> None:
    config = Config()
    n_frontends = config.frontend_processes
    if config.executor_backend == "local" and n_frontends != 1 and not os.environ.get("BEE_FRONTEND_ATTACH"):
        await supervise(config, n_frontends)
        return
    # concrete ports before the executors start: their sandboxes are denied
    # the service's listeners (Landlock TCP layer)
    for attr in ("grpc_listen_addr", "http_listen_addr"):
        host, port = _split_addr(getattr(config, attr))
        if not port and not os.environ.get("BEE_FRONTEND_ATTACH"):
            setattr(config, attr, f"{host}:{_free_port(host)}")
    ctx = ApplicationContext(config)
    stop = _install_stop(asyncio.get_running_loop())
    await ctx.start()
    backend = ctx.code_executor
    if (config.startup_warm_timeout_s > 0 and hasattr(backend, "wait_warm")
            and not os.environ.get("BEE_FRONTEND_ATTACH")):
        await backend.wait_warm(config.startup_warm_timeout_s)
    try:
        await _serve(ctx, stop)
    finally:
        await ctx.close()


# what the self-warm runs: the broker path on GPU slots -- draws, the fused
# and plain reductions, a GEMM, axis sums, a free -- and plain Python on
# CPU-only ones.  Its sandboxes teach the zygotes their trusted copy-on-write
# page sets (csrc/zygote/zygote_loop.cpp "Trust"), so it walks the beekern
# paths user scripts take.
_WARM_GPU = """import beekern as bk
x = bk.random.rand(1 << 16)
s = float(bk.sum(bk.square(x)))
a = bk.random.uniform(-1, 1, (256, 256), dtype="bfloat16")
c = bk.matmul(a, a.T)
r = bk.sum(c, axis=1)
print(s, float(bk.sum(r)), float(bk.max_abs_diff(r, r)))
"""
_WARM_CPU = "print(sum(range(1000)))\n"


async def _self_warm(targets: List[str], total: int, concurrency: int, gpu: bool, max_s: float = 30.0,
                     token: str = "") -> int:
    """``total`` Executes through the replicas' own ports, ``concurrency``
    at a time (closed loop), for at most ``max_s`` seconds, before the
    service says it is ready; returns how many completed.  Failures only end
    the warm-up early."""
    import grpc

    from .models import proto as pb

    chans = [grpc.aio.insecure_channel(t) for t in targets]
    stubs = [pb.CodeInterpreterServiceStub(c) for c in chans]
    budget, done = [total], [0]
    src = _WARM_GPU if gpu else _WARM_CPU

    deadline = time.monotonic() + max_s

    async def client(i: int) -> None:
        stub = stubs[i % len(stubs)]
        while budget[0] > 0 and time.monotonic() < deadline:
            budget[0] -= 1
            try:
                r = await stub.Execute(pb.ExecuteRequest(source_code=src), timeout=120,
                                       metadata=((SELF_WARM_HEADER, token),) if token else None)
            except Exception:  # noqa: BLE001
                budget[0] = 0
                return
            if r.exit_code != 0:
                budget[0] = 0
                return
            done[0] += 1

    try:
        await asyncio.gather(*(client(i) for i in range(concurrency)))
    finally:
        await asyncio.gather(*(c.close() for c in chans), return_exceptions=True)
    return done[0]


def _pin_replica(config: Config, backend, index: int, pid: int) -> None:
    """Replica i runs next to GPU slot i (mod the slot count): its CPU work
    is mostly that slot's sandboxes' RPCs."""
    if (config.numa_affinity or "auto").lower() == "off" or not getattr(backend, "slots", None):
        return
    from .scheduler.topology import slot_cpus

    slot = backend.slots[index % len(backend.slots)]
    cpus = slot_cpus(slot.gpu, slots=[s.gpu for s in backend.slots], factor=config.cpu_quota_pin_factor,
                     quota=config.cpu_quota_override or None)
    if cpus:
        try:
            os.sched_setaffinity(pid, cpus)
        except OSError:
            pass


async def supervise(config: Config, n_frontends: int) -> None:
    """Own the executors; run front-end replicas as child processes."""
    ghost, gport = _split_addr(config.grpc_listen_addr)
    hhost, hport = _split_addr(config.http_listen_addr)
    gport = gport or _free_port(ghost)
    hport = hport or _free_port(hhost)
    config.grpc_listen_addr, config.http_listen_addr = f"{ghost}:{gport}", f"{hhost}:{hport}"
    ctx = ApplicationContext(config)
    backend = ctx.code_executor
    if n_frontends <= 0:
        n_frontends = max(1, min(8, len(getattr(backend, "gpu_ids", None) or [None])))
    # each replica's own gRPC port, picked now so the executors' sandboxes can
    # be denied every listener of the service (Landlock TCP layer)
    replica_ports = [_free_port(ghost) for _ in range(n_frontends)]
    if hasattr(backend, "deny_ports"):
        backend.deny_ports = sorted(set(backend.deny_ports) | {gport, hport, *replica_ports})
    await backend.start()
    if config.startup_warm_timeout_s > 0 and hasattr(backend, "wait_warm"):
        await backend.wait_warm(config.startup_warm_timeout_s)
    env = dict(os.environ)
    # the self-warm's secret: created now, after every executor (and so every
    # sandbox and zygote) started without it, for the replicas alone
    warm_token = secrets.token_hex(16)
    env.update(
        {
            "BEE_SELF_WARM_TOKEN": warm_token,
            "BEE_FRONTEND_ATTACH": backend.attach_spec(),
            "APP_GRPC_LISTEN_ADDR": f"{ghost}:{gport}",
            "APP_HTTP_LISTEN_ADDR": f"{hhost}:{hport}",
            "APP_FRONTEND_PROCESSES": "1",
        }
    )
    children = []
    for i in range(n_frontends):
        e = dict(env, BEE_FRONTEND_INDEX=str(i), BEE_REPLICA_GRPC_PORT=str(replica_ports[i]))
        children.append(subprocess.Popen([sys.executable, "-m", "bee_code_interpreter_fs_amd"], env=e, stdout=subprocess.PIPE))
        _pin_replica(config, backend, i, children[-1].pid)
    loop = asyncio.get_running_loop()
    replicas = []
    for c in children:  # wait until every replica serves
        line = await loop.run_in_executor(None, c.stdout.readline)
        if not line.startswith(b"BEE_SERVICE_READY"):
            raise RuntimeError(f"front-end replica failed to start: {line!r}")
        for part in line.decode().split():
            if part.startswith("replica_grpc="):
                replicas.append(part.split("=", 1)[1])
    if config.startup_self_warm_executions > 0 and replicas:
        t = time.perf_counter()
        n_slots = max(1, len(getattr(backend, "slots", None) or [None]))
        done = await _self_warm(replicas, config.startup_self_warm_executions * n_slots, 8 * n_slots,
                                gpu=bool(getattr(backend, "gpu_ids", None)), max_s=config.startup_self_warm_max_s,
                                token=warm_token)
        logger.info("self-warm: %d Executes through %d replicas in %.2f s", done, len(replicas), time.perf_counter() - t)
    print(
        f"BEE_SERVICE_READY grpc={ghost}:{gport} http={hhost}:{hport} frontends={n_frontends} "
        f"replicas={','.join(replicas)} slots={json.dumps(json.loads(backend.attach_spec()), separators=(',', ':'))}",
        flush=True,
    )
    stop = _install_stop(loop)
    try:
        while not stop.is_set():
            try:
                await asyncio.wait_for(stop.wait(), 2.0)
            except asyncio.TimeoutError:
                pass
            for i, c in enumerate(children):
                if c.poll() is not None and not stop.is_set():  # replica died: replace it
                    e = dict(env, BEE_FRONTEND_INDEX=str(i), BEE_REPLICA_GRPC_PORT=str(replica_ports[i]))
                    children[i] = subprocess.Popen(
                        [sys.executable, "-m", "bee_code_interpreter_fs_amd"], env=e, stdout=subprocess.DEVNULL
                    )
                    _pin_replica(config, backend, i, children[i].pid)
    finally:
        for c in children:
            if c.poll() is None:
                c.send_signal(signal.SIGTERM)
        for c in children:
            try:
                c.wait(timeout=15)
            except subprocess.TimeoutExpired:
                c.kill()
        await ctx.close()


def run() -> None:
    prof_dir = os.environ.get("BEE_FRONTEND_PROFILE")
    if prof_dir and os.environ.get("BEE_FRONTEND_INDEX") is not None:
        # diagnostics: a front-end replica under cProfile, stats dumped at exit
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
        try:
            asyncio.run(main())
        finally:
            prof.disable()
            prof.dump_stats(os.path.join(prof_dir, f"frontend-{os.environ['BEE_FRONTEND_INDEX']}.prof"))
        return
    asyncio.run(main())


if __name__ == "__main__":
    run()
