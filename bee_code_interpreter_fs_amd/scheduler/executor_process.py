"""Launch and talk to one native ``bee-executor`` daemon (one per GPU slot).

The daemon binds a Unix socket (local backend) and prints
``BEE_EXECUTOR_LISTENING <addr>`` once it accepts connections; requests are
HTTP/1.1 JSON over that socket (keep-alive pool, ``uds_http``).
"""

from __future__ import annotations

import asyncio
import logging
import os
import shutil
import signal
import subprocess
import sys
import tempfile
from typing import List, Optional

from .uds_http import Response, UdsHttpClient

logger = logging.getLogger("executor_client")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def default_executor_binary() -> str:
    return os.path.join(ROOT, "bee_code_interpreter_fs_amd", "bin", "bee-executor")


def hbm_interposer_path() -> str:
    return os.path.join(ROOT, "bee_code_interpreter_fs_amd", "lib", "libbee_hbm_quota.so")


def fsmap_path() -> str:
    """libc path shim giving each sandbox its own /workspace (csrc/fsmap)."""
    return os.path.join(ROOT, "bee_code_interpreter_fs_amd", "lib", "libbee_fsmap.so")


class ExecutorProcess:
    def __init__(
        self,
        name: str,
        sandbox_root: str,
        gpus: str,
        target: int,
        binary: Optional[str] = None,
        python: Optional[str] = None,
        warm_gpu: bool = True,
        recursive_scan: bool = False,
        default_timeout: float = 60.0,
        hbm_quota: int = 0,
        max_output: int = 16 << 20,
        max_spawns: int = 8,
        extra_env: Optional[dict] = None,
        use_interposer: bool = True,
        light_target: int = 0,
        broker: bool = False,
        light_zygotes: int = 2,
        extra_args: Optional[List[str]] = None,
        cpus: Optional[List[int]] = None,
    ) -> None:
        self.extra_args = list(extra_args or [])
        self.cpus = list(cpus or [])
        self.light_target = light_target
        self.light_zygotes = light_zygotes
        self.broker = broker
        self.name = name
        self.sandbox_root = os.path.abspath(sandbox_root)
        self.gpus = gpus
        self.target = target
        self.binary = binary or default_executor_binary()
        self.python = python or sys.executable
        self.warm_gpu = warm_gpu
        self.recursive_scan = recursive_scan
        self.default_timeout = default_timeout
        self.hbm_quota = hbm_quota
        self.max_output = max_output
        self.max_spawns = max_spawns
        self.extra_env = dict(extra_env or {})
        self.use_interposer = use_interposer
        self.proc: Optional[subprocess.Popen] = None
        self.address: Optional[str] = None
        self.client: Optional[UdsHttpClient] = None
        self._log_task: Optional[asyncio.Task] = None

    def command(self, socket_path: str) -> List[str]:
        cmd = [
            self.binary,
            "--mode", "pool",
            "--listen", f"unix:{socket_path}",
            "--gpus", self.gpus,
            "--target", str(self.target),
            "--sandbox-root", self.sandbox_root,
            "--python", self.python,
            "--warm-gpu", "1" if self.warm_gpu else "0",
            "--recursive-scan", "1" if self.recursive_scan else "0",
            "--timeout", str(self.default_timeout),
            "--hbm-quota", str(self.hbm_quota),
            "--max-output", str(self.max_output),
            "--max-spawns", str(self.max_spawns),
            "--pythonpath", ROOT,
            "--die-with-parent", "1",
        ]
        lib = os.path.join(ROOT, "bee_code_interpreter_fs_amd", "ops", "lib", "libbeekern.so")
        if self.broker and self.gpus and os.path.exists(lib):
            cmd += ["--broker-lib", lib]
        # light (torch-free) sandboxes: broker-backed on a GPU with a broker,
        # plain CPU-stack sandboxes otherwise
        cmd += ["--light-target", str(self.light_target), "--light-zygotes", str(self.light_zygotes)]
        preload = []
        if os.path.exists(fsmap_path()):
            preload.append(fsmap_path())
        interposer = hbm_interposer_path()
        if self.use_interposer and self.gpus and os.path.exists(interposer):
            preload.append(interposer)
        if preload:
            cmd += ["--preload", ":".join(preload)]
        if self.cpus:
            from .topology import format_cpulist

            cmd += ["--cpus", format_cpulist(self.cpus)]
        return cmd + self.extra_args

    async def start(self, timeout: float = 60.0) -> None:
        if not os.path.exists(self.binary):
            raise RuntimeError(f"bee-executor binary missing at {self.binary}; run the native build first")
        os.makedirs(self.sandbox_root, exist_ok=True)
        run_dir = os.path.join(self.sandbox_root, ".run")
        os.makedirs(run_dir, exist_ok=True)
        sock = os.path.join(run_dir, "executor.sock")
        if len(sock) > 100:  # AF_UNIX path limit (108 bytes)
            sock = os.path.join(tempfile.mkdtemp(prefix="bee-"), "executor.sock")
        env = dict(os.environ)
        env.update(self.extra_env)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.gpus:
            # the daemon's own HIP context (kernel broker) lives on its GPU only
            env["HIP_VISIBLE_DEVICES"] = self.gpus
            # BEE_EXECUTOR_HW_QUEUES: HIP hardware queues behind the kernel
            # broker's per-session streams (GPU_MAX_HW_QUEUES of the daemon
            # only; HIP reads it before main).  Left at the inherited value:
            # on MI355X 2 queues cut the in-sandbox GPU time of 8 concurrent
            # headline Executes from 1.04-1.12 to 0.93-0.96 ms, but moved
            # neither RPS nor p50 beyond box noise (2503 vs 2580, 2437 vs 2329
            # RPS means in two interleaved series; profiles/archive/r2_s3_hw_queues_ab.log)
            if os.environ.get("BEE_EXECUTOR_HW_QUEUES"):
                env["GPU_MAX_HW_QUEUES"] = os.environ["BEE_EXECUTOR_HW_QUEUES"]
        self.log_path = os.path.join(run_dir, "executor.log")
        log = open(self.log_path, "ab")
        try:
            self.proc = subprocess.Popen(
                self.command(sock),
                stdout=subprocess.PIPE,
                stderr=log,  # never inherit our stdio: a lingering daemon would hold pipes open
                stdin=subprocess.DEVNULL,
                env=env,
                start_new_session=True,
            )
        finally:
            log.close()
        loop = asyncio.get_running_loop()
        line = await asyncio.wait_for(loop.run_in_executor(None, self.proc.stdout.readline), timeout)
        text = line.decode().strip()
        if not text.startswith("BEE_EXECUTOR_LISTENING"):
            self.stop()
            raise RuntimeError(f"executor {self.name} failed to start: {text!r}")
        self.address = text.split(" ", 1)[1]
        self.client = UdsHttpClient(self.address[len("unix:") :])
        logger.info("executor %s up at %s (gpus=%r, target=%d)", self.name, self.address, self.gpus, self.target)

    def attach(self, address: str) -> None:
        """Use a daemon started by another process (multi-process front-end)."""
        self.address = address
        self.client = UdsHttpClient(address[len("unix:") :])

    @property
    def socket_path(self) -> Optional[str]:
        return self.address[len("unix:") :] if self.address else None

    def alive(self) -> bool:
        if self.proc is not None:
            return self.proc.poll() is None
        return self.address is not None and os.path.exists(self.socket_path)

    async def post(self, path: str, body: dict, timeout: Optional[float] = None) -> Response:
        assert self.client is not None
        return await self.client.post_json(path, body, timeout)

    async def get_json(self, path: str) -> dict:
        assert self.client is not None
        return await self.client.get_json(path)

    async def wait_ready(self, min_ready: int = 1, timeout: float = 300.0) -> dict:
        """Wait until the pool has ``min_ready`` warm sandboxes."""
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        status: dict = {}
        while loop.time() < deadline:
            status = await self.get_json("/v1/status")
            if status.get("ready", 0) >= min_ready:
                return status
            if not self.alive():
                raise RuntimeError(f"executor {self.name} exited")
            await asyncio.sleep(0.05)
        raise TimeoutError(f"executor {self.name}: pool not ready after {timeout}s: {status}")

    async def close(self) -> None:
        if self.client is not None:
            await self.client.aclose()
            self.client = None
        self.stop()

    def stop(self) -> None:
        if self.proc is None:
            return
        if self.proc.poll() is None:
            try:
                self.proc.send_signal(signal.SIGTERM)
                self.proc.wait(timeout=10)
            except Exception:
                try:
                    os.killpg(self.proc.pid, signal.SIGKILL)
                except OSError:
                    pass
        self.proc = None


def find_python() -> str:
    return sys.executable or shutil.which("python3") or "python3"
