"""SubprocessBackend: a dependency-free reference backend.

Runs each script as a fresh ``python`` process in a throwaway workspace —
the reference executor's semantics without pools, GPUs or the native
daemon.  Used by unit tests of the API layer and as a development fallback
(``APP_EXECUTOR_BACKEND=subprocess``); production uses the local GPU pool.
"""

from __future__ import annotations

import asyncio
import os
import shutil
import signal
import sys
import tempfile
import time
from typing import Dict, Tuple

from ..services.storage import Storage
from ..utils.validation import resolve_logical_path
from .backend import CodeExecutor, ExecuteRequest, ExecutionResult


def _stamp(path: str) -> Tuple[int, int, int, int]:
    st = os.stat(path)
    return (st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns)


def _scan(root: str, recursive: bool) -> Dict[str, Tuple[int, int, int, int]]:
    out = {}
    for dirpath, dirnames, filenames in os.walk(root):
        rel_dir = os.path.relpath(dirpath, root)
        for f in filenames:
            rel = f if rel_dir == "." else os.path.join(rel_dir, f)
            p = os.path.join(dirpath, f)
            if os.path.isfile(p) and not os.path.islink(p):
                out[rel] = _stamp(p)
        if not recursive:
            dirnames.clear()
    return out


class SubprocessBackend(CodeExecutor):
    default_gpus = 0

    def __init__(self, storage: Storage, root: str, default_timeout: float = 60.0, recursive: bool = False) -> None:
        self.storage = storage
        self.root = os.path.abspath(root)
        self.default_timeout = default_timeout
        self.recursive = recursive
        os.makedirs(self.root, exist_ok=True)

    async def run(self, request: ExecuteRequest) -> ExecutionResult:
        t0 = time.perf_counter()
        sandbox = tempfile.mkdtemp(prefix="sbx-", dir=self.root)
        ws = os.path.join(sandbox, "workspace")
        rp = os.path.join(sandbox, "runtime-packages")
        os.makedirs(ws)
        os.makedirs(rp)
        try:
            for logical, obj in request.files.items():
                src = self.storage.path_of(obj)
                if not os.path.isfile(src):
                    raise FileNotFoundError(f"File not found: {obj}")
                dst = resolve_logical_path(logical, ws, rp)
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                shutil.copyfile(src, dst)
            if request.source_file is not None:
                script = resolve_logical_path(request.source_file, ws, rp)
            else:
                script = os.path.join(sandbox, "main.py")
                with open(script, "w") as fh:
                    fh.write(request.source_code or "")
            before = _scan(ws, self.recursive)
            env = dict(os.environ)
            env["PYTHONPATH"] = os.pathsep.join([rp, env.get("PYTHONPATH", "")])
            proc = await asyncio.create_subprocess_exec(
                sys.executable, script, cwd=ws, env=env,
                stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE, start_new_session=True,
            )
            timeout = float(request.timeout or self.default_timeout)
            try:
                out, err = await asyncio.wait_for(proc.communicate(), timeout)
                code = proc.returncode if proc.returncode is not None and proc.returncode >= 0 else -1
                stdout, stderr = out.decode(errors="replace"), err.decode(errors="replace")
            except asyncio.TimeoutError:
                os.killpg(proc.pid, signal.SIGKILL)
                await proc.wait()
                stdout, stderr, code = "", "Execution timed out", -1
            after = _scan(ws, self.recursive)
            files = {}
            for rel, st in after.items():
                if before.get(rel) != st:
                    files["/workspace/" + rel] = self.storage.adopt_file(os.path.join(ws, rel))
            return ExecutionResult(stdout, stderr, code, files, {"total": (time.perf_counter() - t0) * 1e3})
        finally:
            shutil.rmtree(sandbox, ignore_errors=True)
