"""Dependency wiring (lazy singletons), like the reference's
``ApplicationContext`` (`application_context.py:36-126`): config -> logging ->
storage -> executor backend -> custom tools -> gRPC servicer/server -> HTTP app.

Unlike the reference, the backend is started explicitly (``await start()``)
and its background tasks are owned (the reference fire-and-forgets the
initial pool fill, `:83`, dropping its exceptions).
"""

from __future__ import annotations

import asyncio
import contextlib
import logging
import os
from functools import cached_property

import grpc

from .config import Config
from .scheduler.backend import CodeExecutor
from .services.custom_tool_executor import CustomToolExecutor
from .services.grpc_server import GrpcServer
from .services.grpc_servicer import CodeInterpreterServicer
from .services.http_server import create_http_server
from .services.storage import Storage
from .utils.logging import request_id_var, setup_logging

logger = logging.getLogger("application_context")


def _set_non_dumpable() -> None:
    """Sandboxes that share the service's UID (unprivileged deployments) must
    not read its environment (APP_* config, TLS key) or memory through
    /proc/<pid>/: a non-dumpable process needs CAP_SYS_PTRACE for that."""
    try:
        import ctypes

        ctypes.CDLL(None).prctl(4, 0, 0, 0, 0)  # PR_SET_DUMPABLE
    except Exception:
        pass


class ApplicationContext:
    def __init__(self, config: Config = None, setup_log: bool = True) -> None:
        if config is not None:
            self.__dict__["config"] = config
        if setup_log:
            setup_logging(self.config.logging_config, request_id_var)

    @cached_property
    def config(self) -> Config:
        return Config()

    @cached_property
    def file_storage(self) -> Storage:
        os.makedirs(self.config.file_storage_path, exist_ok=True)
        return Storage(self.config.file_storage_path)

    @cached_property
    def code_executor(self) -> CodeExecutor:
        backend = self.config.executor_backend.lower()
        if backend == "local":
            from .scheduler.local_gpu_pool import LocalGpuPoolBackend

            return LocalGpuPoolBackend(self.config, self.file_storage)
        if backend == "kubernetes":
            from .scheduler.kubectl import Kubectl
            from .scheduler.kubernetes_backend import KubernetesBackend

            return KubernetesBackend(
                kubectl=Kubectl(),
                storage=self.file_storage,
                executor_image=self.config.executor_image,
                container_resources=self.config.executor_container_resources,
                executor_pod_spec_extra=self.config.executor_pod_spec_extra,
                queue_target_length=self.config.executor_pod_queue_target_length,
                pod_name_prefix=self.config.executor_pod_name_prefix,
                default_timeout=self.config.default_timeout,
            )
        if backend == "subprocess":
            from .scheduler.subprocess_backend import SubprocessBackend

            return SubprocessBackend(self.file_storage, self.config.sandbox_root, self.config.default_timeout)
        raise ValueError(f"unknown APP_EXECUTOR_BACKEND {self.config.executor_backend!r}")

    @cached_property
    def custom_tool_executor(self) -> CustomToolExecutor:
        return CustomToolExecutor(self.code_executor)

    @cached_property
    def peer_guard(self):
        """Refuses API calls from this node's sandboxes: by the peer socket's
        UID in UID mode, by asking the executors which sandbox holds the peer
        socket when sandboxes share the service's UID (the unprivileged
        deployment); None for other backends or when
        config.api_refuse_sandbox_peers is off."""
        if not self.config.api_refuse_sandbox_peers:
            return None
        from .services.peer_guard import PeerGuard, sandbox_uid_ranges

        ranges = sandbox_uid_ranges(self.config)
        # both checks where both apply: a daemon that could not use its UID
        # range (or sandboxes that share the service's UID) leaves the
        # socket-holder lookup as the control
        holder = getattr(self.code_executor, "socket_holder", None)
        if (self.config.sandbox_isolation or "auto").lower() == "off":
            holder = None
        if not ranges and holder is None:
            return None
        return PeerGuard(ranges, holder_lookup=holder)

    @cached_property
    def grpc_servicer(self) -> CodeInterpreterServicer:
        s = CodeInterpreterServicer(self.code_executor, self.custom_tool_executor)
        s.peer_guard = self.peer_guard
        return s

    @cached_property
    def grpc_server_credentials(self):
        c = self.config
        if not (c.grpc_tls_cert and c.grpc_tls_cert_key and c.grpc_tls_ca_cert):
            return None
        return grpc.ssl_server_credentials(
            private_key_certificate_chain_pairs=[(c.grpc_tls_cert_key, c.grpc_tls_cert)],
            root_certificates=c.grpc_tls_ca_cert,
        )

    @cached_property
    def grpc_server(self) -> GrpcServer:
        return GrpcServer(self.grpc_servicer, self.code_executor.healthy, self.grpc_server_credentials)

    @cached_property
    def http_server(self):
        return create_http_server(self.code_executor, self.custom_tool_executor, self.file_storage,
                                  peer_guard=self.peer_guard)

    async def start(self) -> None:
        _set_non_dumpable()
        await self.code_executor.start()
        ttl = float(self.config.file_storage_ttl_seconds or 0)
        if ttl > 0:
            self._sweeper = asyncio.create_task(self._sweep_storage(ttl))

    async def _sweep_storage(self, ttl: float) -> None:
        """Object retention (``APP_FILE_STORAGE_TTL_SECONDS``):
        sweep a quarter-TTL apart (1 s .. 5 min), off the event loop."""
        period = min(max(ttl / 4, 1.0), 300.0)
        while True:
            try:
                n = await asyncio.to_thread(self.file_storage.sweep, ttl)
                if n:
                    logger.info("storage sweep removed %d object(s) older than %.0f s", n, ttl)
            except Exception:  # keep sweeping; a failed pass is logged, not fatal
                logger.exception("storage sweep failed")
            await asyncio.sleep(period)

    async def close(self) -> None:
        task = self.__dict__.pop("_sweeper", None)
        if task is not None:
            task.cancel()
            with contextlib.suppress(asyncio.CancelledError):
                await task
        await self.code_executor.close()
