"""Executor backend interface shared by the local GPU pool, Kubernetes and
in-process backends.

Parity: the reference's single backend is ``KubernetesCodeExecutor`` with
``execute(source_file, files, timeout) -> Result(stdout, stderr, exit_code,
files)`` (`kubernetes_code_executor.py:48-53,82-161`).  This interface takes
either ``source_code`` (bee-proto / upstream contract, used by gRPC and custom
tools) or ``source_file`` (this fork's HTTP contract) — the fork broke the
former; both work here.
"""

from __future__ import annotations

import abc
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional

from ..utils.validation import ValidationError, check_absolute_path, check_env, check_file_map


@dataclass
class ExecutionResult:
    stdout: str
    stderr: str
    exit_code: int
    files: Dict[str, str]  # logical absolute path -> object id
    timings_ms: Dict[str, float] = field(default_factory=dict)
    gpu_ids: List[int] = field(default_factory=list)


@dataclass
class ExecuteRequest:
    source_code: Optional[str] = None
    source_file: Optional[str] = None
    files: Mapping[str, str] = field(default_factory=dict)
    timeout: Optional[float] = None
    gpus: int = 1  # GPUs for the sandbox (gang size); 0 = CPU-only
    hbm_bytes: Optional[int] = None  # per-request HBM quota override
    nprocs: int = 1  # >1: launch one rank per GPU with torch.distributed env
    env: Mapping[str, str] = field(default_factory=dict)
    # numpy.random draws + numpy calls on them on the GPU (ops/numpy_offload.py);
    # None = the service default (APP_NUMPY_OFFLOAD)
    numpy_offload: Optional[bool] = None
    # internal, never from the wire: the service's own start-up self-warm job
    # (its sandbox's copy-on-write page set is trusted, zygote_loop.cpp "Trust")
    trusted_warm: bool = False

    def validate(self) -> "ExecuteRequest":
        if (self.source_code is None) == (self.source_file is None):
            raise ValidationError("exactly one of source_code / source_file must be given")
        if self.source_file is not None:
            check_absolute_path(self.source_file, "source_file")
        self.files = check_file_map(self.files)
        if self.source_file is not None and self.source_file not in self.files:
            raise ValidationError(f"source_file {self.source_file!r} must be one of the uploaded files")
        if self.timeout is not None and not (0 < float(self.timeout) <= 24 * 3600):
            raise ValidationError("timeout must be in (0, 86400] seconds")
        if not (0 <= int(self.gpus) <= 64):
            raise ValidationError("gpus must be in [0, 64]")
        if int(self.nprocs) < 1 or (int(self.nprocs) > 1 and int(self.nprocs) != max(int(self.gpus), 1)):
            raise ValidationError("nprocs must be 1 or equal to gpus")
        if self.hbm_bytes is not None and int(self.hbm_bytes) < 0:
            raise ValidationError("hbm_bytes must be >= 0")
        self.env = check_env(self.env)
        return self


class CodeExecutor(abc.ABC):
    """What the API layer needs from a backend."""

    async def start(self) -> None:  # pragma: no cover - default no-op
        return None

    async def close(self) -> None:  # pragma: no cover - default no-op
        return None

    @abc.abstractmethod
    async def run(self, request: ExecuteRequest) -> ExecutionResult: ...

    async def execute(
        self,
        source_code: Optional[str] = None,
        source_file: Optional[str] = None,
        files: Optional[Mapping[str, str]] = None,
        timeout: Optional[float] = None,
        gpus: Optional[int] = None,
        hbm_bytes: Optional[int] = None,
        nprocs: int = 1,
        env: Optional[Mapping[str, str]] = None,
        numpy_offload: Optional[bool] = None,
        trusted_warm: bool = False,
    ) -> ExecutionResult:
        req = ExecuteRequest(
            source_code=source_code,
            source_file=source_file,
            files=dict(files or {}),
            timeout=timeout,
            gpus=self.default_gpus if gpus is None else int(gpus),
            hbm_bytes=hbm_bytes,
            nprocs=nprocs,
            env=dict(env or {}),
            numpy_offload=numpy_offload,
            trusted_warm=bool(trusted_warm),
        ).validate()
        return await self.run(req)

    default_gpus: int = 1

    def healthy(self) -> bool:
        return True

    def stats(self) -> dict:
        return {}
