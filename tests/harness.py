"""Run the whole service (gRPC + HTTP + executor backend) in a background
thread, like a deployment, so tests can use plain sync clients the way the
reference's e2e suite does (`test/e2e/test_grpc.py:36-55`)."""

from __future__ import annotations

import asyncio
import os
import threading
import time

import uvicorn

from bee_code_interpreter_fs_amd.application_context import ApplicationContext
from bee_code_interpreter_fs_amd.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ensure_native_executor() -> str:
    from bee_code_interpreter_fs_amd import _build

    _build.build(["bee-executor"], verbose=False)
    return os.path.join(ROOT, "bee_code_interpreter_fs_amd", "bin", "bee-executor")


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ServiceHarness:
    def __init__(self, tmpdir: str, **overrides) -> None:
        # ports picked up front, as a deployment configures them: the
        # executors deny the service's listeners to every sandbox
        base = dict(
            file_storage_path=os.path.join(tmpdir, "files"),
            sandbox_root=os.path.join(tmpdir, "sandboxes"),
            grpc_listen_addr=f"127.0.0.1:{free_port()}",
            http_listen_addr=f"127.0.0.1:{free_port()}",
            gpu_ids=[],
            workers_per_gpu_target=2,
            executor_backend="local",
            # a small numpy-free pool: enough to serve the tests that route
            # there, without 16 more sandboxes per service on the CPU runner
            nano_workers_per_gpu_target=6,
            nano_zygotes_per_gpu=1,
        )
        base.update(overrides)
        self.config = Config(_env={}, **base)
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.ready = threading.Event()
        self.error: BaseException = None
        self.grpc_port = None
        self.http_port = None

    def _run(self) -> None:
        asyncio.set_event_loop(self.loop)
        try:
            self.loop.run_until_complete(self._start())
        except BaseException as e:  # noqa: BLE001
            self.error = e
            self.ready.set()
            return
        self.ready.set()
        self.loop.run_forever()

    async def _start(self) -> None:
        self.ctx = ApplicationContext(self.config, setup_log=False)
        await self.ctx.start()
        if hasattr(self.ctx.code_executor, "wait_ready"):
            await self.ctx.code_executor.wait_ready(120)
        self.grpc_port = self.ctx.grpc_server.bind(self.config.grpc_listen_addr)
        await self.ctx.grpc_server.start()
        self.http = uvicorn.Server(
            uvicorn.Config(self.ctx.http_server, host="127.0.0.1", port=int(self.config.http_listen_addr.rpartition(":")[2]),
                           loop="asyncio", log_level="warning")
        )
        self.http.install_signal_handlers = lambda: None
        self.http_task = asyncio.ensure_future(self.http.serve())
        while not self.http.started:
            await asyncio.sleep(0.01)
        self.http_port = self.http.servers[0].sockets[0].getsockname()[1]

    def start(self) -> "ServiceHarness":
        self.thread.start()
        self.ready.wait(300)
        if self.error:
            raise self.error
        return self

    async def _stop(self) -> None:
        self.http.should_exit = True
        await self.ctx.grpc_server.stop(grace=1)
        await self.http_task
        await self.ctx.close()

    def stop(self) -> None:
        if not self.thread.is_alive():
            return
        fut = asyncio.run_coroutine_threadsafe(self._stop(), self.loop)
        try:
            fut.result(60)
        finally:
            self.loop.call_soon_threadsafe(self.loop.stop)
            self.thread.join(30)

    def call(self, coro, timeout: float = 120):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    @property
    def grpc_target(self) -> str:
        return f"127.0.0.1:{self.grpc_port}"

    @property
    def http_base(self) -> str:
        return f"http://127.0.0.1:{self.http_port}"


def wait_for(pred, timeout=30.0, interval=0.05):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(interval)
    return False


COWSAY_MODULE = '''"""Offline stand-in for the ``cowsay`` distribution (test wheelhouse)."""


def cow(text):
    line = "_" * (len(text) + 2)
    print(" " + line)
    print("| " + text + " |")
    print(" " + "=" * (len(text) + 2))
    print("        \\\\   ^__^")
    print("         \\\\  (oo)\\\\_______")
    print("            (__)\\\\       )\\\\/\\\\")
    print("                ||----w |")
    print("                ||     ||")
'''


def build_test_wheelhouse(directory: str) -> str:
    """Write a pure-Python ``cowsay`` wheel into ``directory``.

    The reference's ``test_ad_hoc_import`` (`test/e2e/test_grpc.py:70-75`)
    needs ``pip install cowsay`` from PyPI; these machines have no package
    index, so the test installs this wheel through the same offline path a
    deployment uses (``APP_WHEELHOUSE``)."""
    import base64
    import hashlib
    import zipfile

    os.makedirs(directory, exist_ok=True)
    name, version = "cowsay", "6.1"
    dist = f"{name}-{version}.dist-info"
    files = {
        f"{name}/__init__.py": COWSAY_MODULE,
        f"{dist}/METADATA": f"Metadata-Version: 2.1\nName: {name}\nVersion: {version}\nSummary: test stand-in\n",
        f"{dist}/WHEEL": "Wheel-Version: 1.0\nGenerator: bee-tests\nRoot-Is-Purelib: true\nTag: py3-none-any\n",
        f"{dist}/top_level.txt": f"{name}\n",
    }
    record = []
    for path, text in files.items():
        data = text.encode()
        digest = base64.urlsafe_b64encode(hashlib.sha256(data).digest()).rstrip(b"=").decode()
        record.append(f"{path},sha256={digest},{len(data)}")
    record.append(f"{dist}/RECORD,,")
    files[f"{dist}/RECORD"] = "\n".join(record) + "\n"
    wheel = os.path.join(directory, f"{name}-{version}-py3-none-any.whl")
    with zipfile.ZipFile(wheel, "w", zipfile.ZIP_DEFLATED) as z:
        for path, text in files.items():
            z.writestr(path, text)
    return directory
