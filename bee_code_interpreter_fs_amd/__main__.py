"""``python -m bee_code_interpreter_fs_amd``: gRPC + HTTP servers in one loop.

Parity with `src/code_interpreter/__main__.py:22-36` (uvicorn + grpc.aio under
one event loop, graceful shutdown); the executor backend (GPU-pinned
sandbox pools) is started before either server accepts requests.
"""

from __future__ import annotations

import asyncio
import signal

import uvicorn

from .application_context import ApplicationContext


def _split_addr(addr: str):
    host, _, port = addr.rpartition(":")
    return host or "0.0.0.0", int(port)


async def main() -> None:
    ctx = ApplicationContext()
    await ctx.start()
    host, port = _split_addr(ctx.config.http_listen_addr)
    http = uvicorn.Server(uvicorn.Config(ctx.http_server, host=host, port=port, loop="asyncio", log_level="warning"))
    http.install_signal_handlers = lambda: None  # handled below
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, stop.set)
    await ctx.grpc_server.start(ctx.config.grpc_listen_addr)
    http_task = asyncio.create_task(http.serve())
    try:
        await stop.wait()
    finally:
        http.should_exit = True
        await ctx.grpc_server.stop(grace=5)
        await http_task
        await ctx.close()


def run() -> None:
    asyncio.run(main())


if __name__ == "__main__":
    run()
