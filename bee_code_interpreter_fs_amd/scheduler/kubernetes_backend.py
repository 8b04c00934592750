"""KubernetesBackend: reference-style single-use executor pods.

Behavioural parity with `services/kubernetes_code_executor.py:40-279`:

* keeps ``executor_pod_queue_target_length`` Ready pods; each request takes
  one (spawning synchronously if none is ready) and the pod is deleted after
  use; the queue is refilled after every take (`:163-201`, `:263-279`);
* pods are labelled ``app=code-executor``, owned by the service pod
  (``ownerReferences`` from ``$HOSTNAME``) so Kubernetes garbage-collects
  them, carry ``executor_container_resources`` (e.g. ``amd.com/gpu: 1`` for
  an MI355X) and ``executor_pod_spec_extra`` (runtimeClass, /dev/shm ...);
* spawn: ``kubectl create -f -`` + ``kubectl wait --for=condition=Ready
  --timeout=60s``, delete on failure, ``RuntimeError`` retried 3x with
  exponential 4-10 s backoff (`:203-261`);
* per request: objects are streamed to ``PUT /{workspace|runtime-packages}/
  <path>`` on the pod, ``POST /execute``, changed files streamed back into
  the object store.

Fixes over the reference: the pod runs the native ``bee-executor --mode pod``
which accepts ``source_code`` directly (gRPC/custom-tool paths work), the
request ``timeout`` is forwarded and enforced in the pod, spawn concurrency
is bounded, and background tasks are owned and their failures logged.
"""

from __future__ import annotations

import asyncio
import collections
import logging
import os
import random
import string
import time
from contextlib import asynccontextmanager
from typing import Dict, Optional

import httpx

from ..services.storage import Storage
from ..utils.retry import async_retry
from ..utils.validation import split_logical_path
from .backend import CodeExecutor, ExecuteRequest, ExecutionResult
from .kubectl import Kubectl

logger = logging.getLogger("kubernetes_code_executor")

EXECUTOR_PORT = 8000


class KubernetesBackend(CodeExecutor):
    default_gpus = 0

    def __init__(
        self,
        kubectl: Kubectl,
        storage: Storage,
        executor_image: str,
        container_resources: dict,
        executor_pod_spec_extra: dict,
        queue_target_length: int = 5,
        pod_name_prefix: str = "code-executor-",
        default_timeout: float = 60.0,
        max_concurrent_spawns: int = 16,
        retry_sleep=asyncio.sleep,
    ) -> None:
        self.kubectl = kubectl
        self.storage = storage
        self.executor_image = executor_image
        self.container_resources = container_resources
        self.executor_pod_spec_extra = executor_pod_spec_extra
        self.queue_target_length = queue_target_length
        self.pod_name_prefix = pod_name_prefix
        self.default_timeout = default_timeout
        self.queue: collections.deque = collections.deque()
        self.spawning = 0
        self.self_pod: Optional[dict] = None
        self._spawn_sem = asyncio.Semaphore(max_concurrent_spawns)
        self._tasks: set = set()
        self._retry_sleep = retry_sleep
        self._spawn = async_retry((RuntimeError,), 3, sleep=retry_sleep)(self._spawn_once)

    # ---- background task ownership --------------------------------------------------
    def _background(self, coro, what: str) -> None:
        task = asyncio.ensure_future(coro)
        self._tasks.add(task)

        def done(t: asyncio.Task) -> None:
            self._tasks.discard(t)
            if not t.cancelled() and t.exception() is not None:
                logger.error("%s failed: %s", what, t.exception())

        task.add_done_callback(done)

    async def start(self) -> None:
        self._background(self.fill_queue(), "initial pod queue fill")

    async def close(self) -> None:
        for t in list(self._tasks):
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)

    # ---- pod pool -----------------------------------------------------------------------
    async def fill_queue(self) -> None:
        need = self.queue_target_length - len(self.queue) - self.spawning
        if need <= 0:
            return
        logger.info("Extending executor pod queue: target %d, ready %d, spawning %d, to spawn %d",
                    self.queue_target_length, len(self.queue), self.spawning, need)
        self.spawning += need

        async def one():
            try:
                self.queue.append(await self._spawn())
            except Exception:
                logger.exception("Failed to spawn executor pod")
            finally:
                self.spawning -= 1

        await asyncio.gather(*(one() for _ in range(need)))

    def pod_manifest(self, name: str) -> dict:
        meta: Dict = {"name": name, "labels": {"app": "code-executor"}}
        if self.self_pod:
            meta["ownerReferences"] = [
                {
                    "apiVersion": "v1",
                    "kind": "Pod",
                    "name": self.self_pod["metadata"]["name"],
                    "uid": self.self_pod["metadata"]["uid"],
                    "controller": True,
                    "blockOwnerDeletion": False,
                }
            ]
        return {
            "apiVersion": "v1",
            "kind": "Pod",
            "metadata": meta,
            "spec": {
                "containers": [
                    {
                        "name": "executor",
                        "image": self.executor_image,
                        "args": ["--mode", "pod", "--listen", f"0.0.0.0:{EXECUTOR_PORT}"],
                        "resources": self.container_resources,
                        "ports": [{"containerPort": EXECUTOR_PORT}],
                    }
                ],
                **self.executor_pod_spec_extra,
            },
        }

    async def _spawn_once(self) -> dict:
        async with self._spawn_sem:
            if self.self_pod is None and os.environ.get("HOSTNAME"):
                try:
                    self.self_pod = await self.kubectl.get("pod", os.environ["HOSTNAME"])
                except RuntimeError:
                    logger.warning("not running in a pod; executor pods get no ownerReferences")
                    self.self_pod = {}
            name = self.pod_name_prefix + "".join(random.choices(string.ascii_lowercase + string.digits, k=6))
            try:
                await self.kubectl.create(filename="-", input=self.pod_manifest(name))
                return await self.kubectl.wait("pod", name, _for="condition=Ready", timeout="60s")
            except Exception as e:
                try:
                    await self.kubectl.delete("pod", name, wait="false")
                except Exception:
                    pass
                raise RuntimeError(f"Failed to spawn the pod: {e}") from e

    @asynccontextmanager
    async def executor_pod(self):
        pod = self.queue.popleft() if self.queue else await self._spawn()
        self._background(self.fill_queue(), "pod queue refill")
        name = pod["metadata"]["name"]
        try:
            logger.info("Grabbing executor pod %s", name)
            yield pod
        finally:
            logger.info("Removing used executor pod %s", name)
            self._background(self.kubectl.delete("pod", name, wait="false"), f"delete pod {name}")

    # ---- execution ----------------------------------------------------------------------
    async def run(self, request: ExecuteRequest) -> ExecutionResult:
        attempt = async_retry((RuntimeError,), 3, sleep=self._retry_sleep)(self._run_once)
        return await attempt(request)

    async def _run_once(self, request: ExecuteRequest) -> ExecutionResult:
        t0 = time.perf_counter()
        timeout = float(request.timeout or self.default_timeout)
        async with self.executor_pod() as pod, httpx.AsyncClient(timeout=timeout + 30) as client:
            port = int(pod["metadata"].get("annotations", {}).get("bee.executor/port", EXECUTOR_PORT))
            base = f"http://{pod['status']['podIP']}:{port}"

            async def upload(path: str, obj: str):
                root, rel = split_logical_path(path)
                async with self.storage.reader(obj) as r:
                    resp = await client.put(f"{base}{root}/{rel}", content=r.iter_chunks())
                if resp.status_code >= 400:
                    raise RuntimeError(f"upload of {path} failed: {resp.status_code} {resp.text}")

            await asyncio.gather(*(upload(p, o) for p, o in request.files.items()))
            body = {"timeout": timeout}
            if request.numpy_offload:
                body["numpy_offload"] = True  # the pod's executor hands it to the sandbox
            if request.source_file is not None:
                body["source_file"] = request.source_file
            else:
                body["source_code"] = request.source_code
            resp = await client.post(f"{base}/execute", json=body)
            if resp.status_code != 200:
                raise RuntimeError(f"executor pod error {resp.status_code}: {resp.text}")
            data = resp.json()

            async def download(path: str):
                rel = path[len("/workspace/") :] if path.startswith("/workspace/") else path.lstrip("/")
                async with self.storage.writer() as w, client.stream("GET", f"{base}/workspace/{rel}") as r:
                    r.raise_for_status()
                    async for chunk in r.aiter_bytes():
                        await w.write(chunk)
                return path, w.hash

            files = dict(await asyncio.gather(*(download(p) for p in data.get("files", []))))
        return ExecutionResult(
            stdout=data.get("stdout", ""),
            stderr=data.get("stderr", ""),
            exit_code=int(data.get("exit_code", -1)),
            files=files,
            timings_ms={"service_total": (time.perf_counter() - t0) * 1e3},
        )

    def stats(self) -> dict:
        return {"backend": "kubernetes", "ready_pods": len(self.queue), "spawning": self.spawning}
