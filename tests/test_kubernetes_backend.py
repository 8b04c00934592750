"""Kubernetes backend without a cluster: a fake ``kubectl`` whose "pods" are
real ``bee-executor --mode pod`` processes on localhost, so the whole
reference flow (create -> wait Ready -> PUT files -> POST /execute -> GET
changed files -> delete) runs against the native pod-mode server."""

import asyncio
import json
import os
import socket
import subprocess
import time

import httpx
import pytest

from bee_code_interpreter_fs_amd.scheduler.kubectl import Kubectl
from bee_code_interpreter_fs_amd.scheduler.kubernetes_backend import KubernetesBackend
from bee_code_interpreter_fs_amd.services.storage import Storage

from .harness import ROOT, ensure_native_executor


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeKubectl(Kubectl):
    """Records argv; 'creates' pods as local pod-mode executors."""

    def __init__(self, root):
        super().__init__(namespace="test")
        self.root = root
        self.calls = []
        self.pods = {}

    async def _exec(self, argv, stdin):
        self.calls.append(argv)
        verb = argv[0]
        if verb == "get":
            return 1, b"", b"pods not found"
        if verb == "create":
            manifest = json.loads(stdin)
            name = manifest["metadata"]["name"]
            port = free_port()
            ws = os.path.join(self.root, name, "workspace")
            rp = os.path.join(self.root, name, "runtime-packages")
            proc = subprocess.Popen(
                [
                    os.path.join(ROOT, "bee_code_interpreter_fs_amd", "bin", "bee-executor"),
                    "--mode", "pod", "--listen", f"127.0.0.1:{port}",
                    "--workspace", ws, "--runtime-packages", rp,
                    "--sandbox-root", os.path.join(self.root, name, "sb"),
                    "--pythonpath", ROOT, "--die-with-parent", "1",
                ],
                stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=dict(os.environ, BEE_PRELOAD="numpy"),
            )
            proc.stdout.readline()
            self.pods[name] = (proc, port, manifest)
            return 0, json.dumps(manifest).encode(), b""
        if verb == "wait":
            name = argv[2]
            proc, port, manifest = self.pods[name]
            pod = dict(manifest)
            pod["metadata"] = dict(manifest["metadata"], annotations={"bee.executor/port": str(port)})
            pod["status"] = {"podIP": "127.0.0.1", "phase": "Running"}
            # Ready = the in-pod sandbox is warm
            for _ in range(400):
                try:
                    st = httpx.get(f"http://127.0.0.1:{port}/v1/status", timeout=2).json()
                    if st["ready"] >= 1:
                        break
                except httpx.HTTPError:
                    pass
                await asyncio.sleep(0.05)
            return 0, json.dumps(pod).encode(), b""
        if verb == "delete":
            name = argv[2]
            if name in self.pods:
                proc = self.pods.pop(name)[0]
                proc.terminate()
                proc.wait(10)
            return 0, b"", b""
        return 1, b"", b"unsupported"

    def shutdown(self):
        for proc, _, _ in self.pods.values():
            proc.terminate()
            proc.wait(10)


def test_kubectl_argv_building():
    k = Kubectl(namespace="ns", context=None)
    assert k.build_args("delete", "pod", "p1", now=True, grace_period=0) == ["delete", "pod", "p1", "--namespace=ns", "--now", "--grace-period=0"]
    assert k.build_args("exec", "p", "--", "ls", "-l", container="c") == ["exec", "p", "--namespace=ns", "--container=c", "--", "ls", "-l"]
    assert k.build_args("wait", "pod", "x", _for="condition=Ready") == ["wait", "pod", "x", "--namespace=ns", "--for=condition=Ready"]
    with pytest.raises(AttributeError):
        k.frobnicate


def test_kubernetes_backend_end_to_end(tmp_path):
    ensure_native_executor()
    kube = FakeKubectl(str(tmp_path / "pods"))
    storage = Storage(str(tmp_path / "files"))

    async def nosleep(_):
        return None

    async def go():
        be = KubernetesBackend(
            kube, storage, "img:latest", {"limits": {"amd.com/gpu": 1}}, {"runtimeClassName": "kata"},
            queue_target_length=1, retry_sleep=nosleep,
        )
        await be.start()
        try:
            data = await storage.write(b"hello from storage")
            r = await be.execute(
                source_code="print(open('in/data.txt').read())\nopen('out.txt','w').write('ok')",
                files={"/workspace/in/data.txt": data},
            )
            assert r.exit_code == 0, r.stderr
            assert r.stdout == "hello from storage\n"
            assert set(r.files) == {"/workspace/out.txt"}
            assert await storage.read(r.files["/workspace/out.txt"]) == b"ok"
            r2 = await be.execute(source_code="import time; time.sleep(5)", timeout=1)
            assert r2.exit_code == -1 and "Execution timed out" in r2.stderr
        finally:
            await be.close()
            kube.shutdown()

    asyncio.run(go())
    creates = [c for c in kube.calls if c[0] == "create"]
    assert creates and all("--namespace=test" in c and "--filename=-" in c for c in creates)
    waits = [c for c in kube.calls if c[0] == "wait"]
    assert waits and "--for=condition=Ready" in waits[0] and "--timeout=60s" in waits[0]
    assert any(c[0] == "delete" for c in kube.calls)  # single-use pods are deleted


def test_pod_manifest_shape(tmp_path):
    be = KubernetesBackend(Kubectl(), Storage(str(tmp_path)), "img", {"limits": {"amd.com/gpu": 1}}, {"runtimeClassName": "kata"})
    be.self_pod = {"metadata": {"name": "svc", "uid": "u1"}}
    m = be.pod_manifest("code-executor-abc123")
    assert m["metadata"]["labels"] == {"app": "code-executor"}
    assert m["metadata"]["ownerReferences"][0]["uid"] == "u1"
    c = m["spec"]["containers"][0]
    assert c["name"] == "executor" and c["ports"] == [{"containerPort": 8000}]
    assert c["resources"] == {"limits": {"amd.com/gpu": 1}}
    assert m["spec"]["runtimeClassName"] == "kata"
