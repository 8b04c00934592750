"""Sandbox isolation (runtime/jail.py, csrc/jail/jail.cpp, the executor's
peer checks) end to end on CPU, against hostile user code.

The reference isolates each execution in its own pod as a non-root UID
(`kubernetes_code_executor.py:220-253`, `executor/Dockerfile:91-98`): user
code cannot see the file-object store, other executions or the service.
These tests run attacks from inside a sandbox and assert that each one
fails while the service keeps working:

* ``jailed``: Landlock + seccomp + scoping only (the sandboxes keep the
  service's UID) -- what an unprivileged deployment (and the MI355X box,
  which runs as an ordinary user) gets;
* ``uid``: the service runs as root, so every sandbox additionally gets a
  UID/GID of its own, ``RLIMIT_NPROC`` per UID and a kill sweep of the UID.
  The sandbox UIDs must be able to walk to the interpreter and package, so
  that service runs from a copy of the package under a world-searchable
  directory (this repository sits in a 0700 ``$HOME`` here, where the
  executor itself falls back to the ``jailed`` level -- see
  ``test_uid_mode_falls_back_on_private_layout``).
"""

from __future__ import annotations

import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import textwrap
import threading
import time

import httpx
import pytest

from .harness import ServiceHarness, ensure_native_executor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _jail_built() -> bool:
    from bee_code_interpreter_fs_amd.runtime import jail

    return jail.available() and jail.probe().get("landlock_abi", 0) >= 6


pytestmark = pytest.mark.skipif(not _jail_built(), reason="native jail not built or Landlock ABI < 6")


# ---- services under test -------------------------------------------------------------


class InProcess:
    """Landlock/seccomp-only service (this checkout lives under a 0700 $HOME)."""

    def __init__(self, tmp: str, **overrides) -> None:
        ensure_native_executor()
        kw = dict(gpu_ids=[], workers_per_gpu_target=2, sandbox_isolation="on", sandbox_memory_bytes=2 * 1024**3,
                  sandbox_max_processes=64, sandbox_net_layer=True, sandbox_network="open")
        kw.update(overrides)
        self.h = ServiceHarness(tmp, **kw)
        self.h.start()
        self.storage = self.h.ctx.file_storage.storage_path
        self.sandbox_root = self.h.config.sandbox_root
        self.service_pid = os.getpid()
        self.http = httpx.Client(base_url=self.h.http_base, timeout=120)
        self.grpc_target = self.h.grpc_target

    def executor_socket(self) -> str:
        return self.h.ctx.code_executor.slots[0].executor.socket_path

    def executor_status(self) -> dict:
        return self.h.call(self.h.ctx.code_executor.slots[0].executor.get_json("/v1/status"))

    def stop(self) -> None:
        self.http.close()
        self.h.stop()


UID_DRIVER = textwrap.dedent(
    """
    import json, os, sys, time
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from tests.harness import ServiceHarness
    tmp = sys.argv[1]
    kw = dict(gpu_ids=[], workers_per_gpu_target=2, sandbox_isolation="on",
              sandbox_memory_bytes=2 * 1024**3, sandbox_max_processes=64, sandbox_net_layer=True,
              sandbox_network="open", sandbox_uid_base=1500000000, sandbox_uid_count=64)
    kw.update(json.loads(sys.argv[2]) if len(sys.argv) > 2 else {})
    h = ServiceHarness(tmp, **kw)
    h.start()
    ex = h.ctx.code_executor.slots[0].executor
    print(json.dumps({"http": h.http_base, "grpc": h.grpc_target, "storage": h.ctx.file_storage.storage_path,
                      "sandbox_root": h.config.sandbox_root, "socket": ex.socket_path}), flush=True)
    sys.stdin.read()  # until the test closes our stdin
    h.stop()
    """
)


class UidService:
    """Service as root with per-sandbox UIDs, run from a world-searchable copy."""

    def __init__(self, **overrides) -> None:
        ensure_native_executor()
        self.base = tempfile.mkdtemp(prefix="bee-uid-")
        os.chmod(self.base, 0o755)
        tree = os.path.join(self.base, "tree")
        shutil.copytree(os.path.join(ROOT, "bee_code_interpreter_fs_amd"), os.path.join(tree, "bee_code_interpreter_fs_amd"),
                        ignore=shutil.ignore_patterns("__pycache__"), symlinks=True)
        os.makedirs(os.path.join(tree, "tests"))
        for f in ("__init__.py", "harness.py"):
            shutil.copy(os.path.join(ROOT, "tests", f), os.path.join(tree, "tests", f))
        with open(os.path.join(tree, "uid_driver.py"), "w") as fh:
            fh.write(UID_DRIVER)
        for d, dirs, files in os.walk(self.base):
            os.chmod(d, 0o755)
        svc = os.path.join(self.base, "svc")
        os.makedirs(svc)
        env = dict(os.environ)
        env.pop("PYTHONPATH", None)
        self.proc = subprocess.Popen([sys.executable, os.path.join(tree, "uid_driver.py"), svc, json.dumps(overrides)],
                                     cwd=tree, env=env,
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                     text=True, start_new_session=True)
        line = self.proc.stdout.readline()
        if not line:
            raise RuntimeError("uid service failed to start")
        info = json.loads(line)
        self.storage, self.sandbox_root = info["storage"], info["sandbox_root"]
        self.grpc_target = info["grpc"]
        self._socket = info["socket"]
        self.service_pid = self.proc.pid
        self.http = httpx.Client(base_url=info["http"], timeout=120)

    def executor_socket(self) -> str:
        return self._socket

    def executor_status(self) -> dict:
        # the control socket speaks HTTP/1.1; the test process runs as root,
        # outside every sandbox
        with socket.socket(socket.AF_UNIX) as s:
            s.settimeout(10)
            s.connect(self._socket)
            s.sendall(b"GET /v1/status HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            data = b""
            while True:
                chunk = s.recv(65536)
                if not chunk:
                    break
                data += chunk
        return json.loads(data.split(b"\r\n\r\n", 1)[1])

    def stop(self) -> None:
        self.http.close()
        try:
            self.proc.stdin.close()
            self.proc.wait(60)
        except Exception:
            os.killpg(self.proc.pid, signal.SIGKILL)
        shutil.rmtree(self.base, ignore_errors=True)


@pytest.fixture(scope="module", params=["jailed", "uid"])
def svc(request, tmp_path_factory):
    if request.param == "uid":
        if os.geteuid() != 0:
            pytest.skip("per-sandbox UIDs need a root service")
        s = UidService()
    else:
        s = InProcess(str(tmp_path_factory.mktemp("iso")))
    s.mode = request.param
    yield s
    s.stop()


def run(svc, code: str, files=None, timeout: float = 60) -> dict:
    body = {"source_code": textwrap.dedent(code), "files": files or {}, "timeout": timeout}
    r = svc.http.post("/v1/execute", json=body, timeout=timeout + 60)
    assert r.status_code == 200, r.text
    return r.json()


def upload(svc, data: bytes) -> str:
    r = svc.http.put("/v1/files", files={"file": ("f", data)})
    assert r.status_code == 200, r.text
    return r.json()["hash"]


# ---- tests -----------------------------------------------------------------------------


def test_status_reports_isolation(svc):
    iso = svc.executor_status()["isolation"]
    assert iso["jail"] is True
    assert iso["uid_mode"] is (svc.mode == "uid"), iso


def test_identity(svc):
    r = run(svc, "import os; print(os.getuid(), os.getgid())")
    uid = int(r["stdout"].split()[0])
    if svc.mode == "uid":
        assert 1500000000 <= uid < 1500000064, r
    else:
        assert uid == os.geteuid()


def test_sandbox_process_group_and_session(svc):
    """A sandbox leads its own process group (the executor's kill and the
    broker's peer lookup go by it) and session, with no controlling
    terminal: there is no tty to open or inject into, and the group leader
    cannot setsid() itself out of its group."""
    r = run(svc, """
        import os
        print(os.getpgrp() == os.getpid(), os.getsid(0) == os.getpid())
        try:
            os.setsid(); print("setsid ok")
        except OSError as e:
            print("setsid", e.errno)
        try:
            os.open("/dev/tty", os.O_RDWR); print("tty ok")
        except OSError as e:
            print("tty", e.errno)
    """)
    lines = r["stdout"].split("\n")
    assert lines[0] == "True True", r
    assert lines[1] == "setsid 1", r  # EPERM
    assert lines[2].startswith("tty ") and lines[2] != "tty ok", r


def test_cannot_read_another_users_object(svc):
    secret = b"TOP-SECRET-OF-USER-A"
    oid = upload(svc, secret)
    # another user's execution that writes an output object too
    a = run(svc, "open('/workspace/out.txt', 'w').write('SECRET-OUTPUT-OF-USER-A')")
    out_oid = a["files"]["/workspace/out.txt"]
    r = run(svc, f"""
        import os, glob
        store = {svc.storage!r}
        for attempt in (lambda: open(os.path.join(store, {oid!r})).read(),
                        lambda: open(os.path.join(store, {out_oid!r})).read(),
                        lambda: os.listdir(store),
                        lambda: os.listdir(os.path.dirname(store)),
                        lambda: os.listdir({svc.sandbox_root!r}),
                        lambda: glob.glob({svc.sandbox_root!r} + '/**/*', recursive=True) or 1 / 0):
            try:
                print("LEAK", attempt())
            except (OSError, ZeroDivisionError) as e:
                print("denied", type(e).__name__)
    """)
    assert r["exit_code"] == 0, r
    assert "LEAK" not in r["stdout"] and "SECRET" not in r["stdout"], r["stdout"]
    assert r["stdout"].count("denied") == 6, r["stdout"]
    # the owner still gets both objects back
    assert svc.http.get(f"/v1/files/{oid}").content == secret
    assert svc.http.get(f"/v1/files/{out_oid}").content == b"SECRET-OUTPUT-OF-USER-A"


def test_cannot_read_service_environment(svc):
    r = run(svc, f"""
        import os
        for pid in ({svc.service_pid}, os.getppid(), 1):
            for leaf in ("environ", "cwd", "root", "fd", "mem", "maps"):
                p = f"/proc/{{pid}}/{{leaf}}"
                try:
                    if leaf == "fd":  # where the descriptors point (numbers alone say nothing)
                        data = [os.readlink(p + "/" + n) for n in os.listdir(p)]
                    elif leaf in ("cwd", "root"):
                        data = os.listdir(p)
                    else:
                        data = open(p, "rb").read(64)
                    print("LEAK", p, data[:3])
                except OSError as e:
                    pass
        print("own environ ok", len(open("/proc/self/environ", "rb").read()) > 0)
    """)
    assert r["exit_code"] == 0, r
    assert "LEAK" not in r["stdout"], r["stdout"]
    assert "own environ ok True" in r["stdout"]


def test_cannot_drive_the_executor(svc):
    """The control socket stages arbitrary host paths into a workspace: a
    sandbox that reached it could read any file as the service."""
    r = run(svc, f"""
        import json, socket
        body = json.dumps({{"source_code": "print(open('/workspace/x').read())",
                            "files": {{"/workspace/x": "/etc/hostname"}}}}).encode()
        req = (b"POST /v1/execute HTTP/1.1\\r\\nHost: x\\r\\nContent-Type: application/json\\r\\n"
               b"Content-Length: " + str(len(body)).encode() + b"\\r\\n\\r\\n" + body)
        try:
            s = socket.socket(socket.AF_UNIX)
            s.settimeout(10)
            s.connect({svc.executor_socket()!r})
            s.sendall(req)
            resp = s.recv(65536)
            print("RESPONSE", resp[:80])
        except OSError as e:
            print("denied", type(e).__name__)
    """)
    assert r["exit_code"] == 0, r
    # refused at connect (UID mode: 0600 socket) or closed unanswered (peer check)
    assert "denied" in r["stdout"] or "RESPONSE b''" in r["stdout"], r["stdout"]


def test_cannot_signal_or_trace_other_processes(svc):
    token = f"/dev/shm/bee-iso-{os.getpid()}-{svc.mode}"
    victim = f"""
        import os, time
        open({token!r}, "w").write(str(os.getpid()))
        time.sleep(4)
        print("victim alive")
    """
    results = {}
    t = threading.Thread(target=lambda: results.setdefault("victim", run(svc, victim)))
    t.start()
    try:
        r = run(svc, f"""
            import ctypes, os, signal, time
            for _ in range(200):
                if os.path.exists({token!r}) and open({token!r}).read():
                    break
                time.sleep(0.02)
            victim = int(open({token!r}).read())
            libc = ctypes.CDLL(None, use_errno=True)
            for pid in (victim, os.getppid(), {svc.service_pid}):
                try:
                    os.kill(pid, signal.SIGKILL)
                    print("KILLED", pid)
                except PermissionError:
                    print("kill denied")
                # PTRACE_ATTACH
                rc = libc.ptrace(16, pid, None, None)
                print("ptrace", rc, ctypes.get_errno())
            # own children stay killable
            child = os.fork()
            if child == 0:
                time.sleep(30)
                os._exit(0)
            os.kill(child, signal.SIGKILL)
            print("own child", os.waitpid(child, 0)[1])
        """)
    finally:
        t.join(60)
        try:
            os.unlink(token)
        except OSError:
            pass
    assert r["exit_code"] == 0, r
    assert "KILLED" not in r["stdout"] and r["stdout"].count("kill denied") == 3, r["stdout"]
    assert r["stdout"].count("ptrace -1 1") == 3, r["stdout"]  # EPERM
    assert "own child 9" in r["stdout"], r["stdout"]
    assert results["victim"]["exit_code"] == 0 and "victim alive" in results["victim"]["stdout"], results


def test_private_tmp(svc):
    r = run(svc, """
        import os, tempfile
        open("/tmp/scratch.txt", "w").write("mine")
        print(sorted(os.listdir("/tmp")), open("/tmp/scratch.txt").read())
        with tempfile.NamedTemporaryFile() as f:
            print("tempfile ok")
    """)
    assert r["exit_code"] == 0, r
    assert "scratch.txt" in r["stdout"] and "mine" in r["stdout"], r["stdout"]
    assert not os.path.exists("/tmp/scratch.txt")
    # the next sandbox starts with an empty /tmp
    r2 = run(svc, "import os; print(os.path.exists('/tmp/scratch.txt'))")
    assert r2["stdout"].strip() == "False", r2


def test_memory_cap_contains_a_huge_allocation(svc):
    r = run(svc, "x = bytearray(100 * 1024**3)\nprint('ALLOCATED')")
    assert r["exit_code"] != 0 and "MemoryError" in r["stderr"], r
    assert "ALLOCATED" not in r["stdout"]
    assert run(svc, "print(6 * 7)")["stdout"] == "42\n"


def test_fork_bomb_is_contained(svc):
    if svc.mode != "uid":
        pytest.skip("RLIMIT_NPROC of a sandbox UID; without one the executor monitor bounds it (test_containment_cpu.py)")
    t0 = time.time()
    r = run(svc, """
        import os, time
        print(os.getuid(), flush=True)
        n = 0
        try:
            while True:
                if os.fork() == 0:
                    time.sleep(60)
                    os._exit(0)
                n += 1
        except OSError as e:
            print("refused after", n, type(e).__name__)
    """, timeout=60)
    assert r["exit_code"] == 0 and "refused after" in r["stdout"], r
    uid1, line = r["stdout"].splitlines()[:2]
    n = int(line.split()[2])
    assert 10 < n < 64, r["stdout"]
    # the classic bomb: every process forks until refused, then dies
    r = run(svc, "import os\nprint(os.getuid(), flush=True)\nwhile True:\n    os.fork()\n", timeout=60)
    assert r["exit_code"] != 0
    uid2 = r["stdout"].split()[0]
    assert time.time() - t0 < 100
    # nothing survives under those sandboxes' UIDs (the sleeping children
    # included), and the service is healthy
    def leftovers():
        n = 0
        for pid in os.listdir("/proc"):
            if pid.isdigit():
                try:
                    if os.stat(f"/proc/{pid}").st_uid in (int(uid1), int(uid2)):
                        n += 1
                except OSError:
                    pass
        return n

    deadline = time.time() + 10
    while leftovers() and time.time() < deadline:
        time.sleep(0.2)
    assert leftovers() == 0
    assert run(svc, "print(6 * 7)")["stdout"] == "42\n"


def test_outputs_and_inputs_still_work(svc):
    oid = upload(svc, b"1,2,3\n")
    r = run(svc, """
        import numpy as np
        data = np.loadtxt('/workspace/in.csv', delimiter=',')
        open('/workspace/sum.txt', 'w').write(str(data.sum()))
        import os; os.makedirs('/workspace/sub', exist_ok=True)
        print(sorted(os.listdir('/workspace')))
    """, files={"/workspace/in.csv": oid})
    assert r["exit_code"] == 0, r
    got = svc.http.get(f"/v1/files/{r['files']['/workspace/sum.txt']}").content
    assert got == b"6.0"


def test_uid_mode_falls_back_on_private_layout(tmp_path):
    """A service root under a directory other UIDs cannot search keeps the
    jail but not the UID switch, and says why."""
    if os.geteuid() != 0:
        pytest.skip("needs root")
    private = tmp_path / "private"
    private.mkdir(mode=0o700)
    os.chmod(private, 0o700)
    ensure_native_executor()
    h = ServiceHarness(str(private), gpu_ids=[], workers_per_gpu_target=1, sandbox_isolation="on",
                       sandbox_uid_base=1500000100, sandbox_uid_count=8)
    h.start()
    try:
        st = h.call(h.ctx.code_executor.slots[0].executor.get_json("/v1/status"))
        assert st["isolation"]["uid_mode"] is False and "not searchable" in st["isolation"]["note"], st
        r = h.call(h.ctx.code_executor.execute(source_code="print('ok')", timeout=30), timeout=60)
        assert r.stdout == "ok\n"
    finally:
        h.stop()


def test_request_env_cannot_switch_the_jail_off(svc):
    """The daemon's own floor under the service's env allow-list: a request
    that reaches the control socket with BEE_JAIL*=0 still gets a jailed
    sandbox; harmless variables pass."""
    if svc.mode != "jailed":
        pytest.skip("needs the in-process harness (executor client)")
    ex = svc.h.ctx.code_executor.slots[0].executor
    body = {"source_code": f"import os\ntry:\n    os.listdir({svc.storage!r}); print('LEAK')\nexcept OSError:\n    print('denied')\n"
                           "print(os.environ.get('USER_X'), os.environ.get('BEE_JAIL_LANDLOCK'))\n",
            "env": {"BEE_JAIL": "0", "BEE_JAIL_LANDLOCK": "0", "BEE_JAIL_SECCOMP": "0", "LD_PRELOAD": "", "USER_X": "1"},
            "timeout": 60}
    resp = svc.h.call(ex.post("/v1/execute", body))
    out = resp.json()
    assert out["stdout"].split() == ["denied", "1", "None"], out


def test_service_ports_are_unreachable_from_sandboxes(svc):
    """APP_SANDBOX_NET_LAYER: the service's own TCP listeners (gRPC, HTTP)
    are denied to every sandbox by a Landlock network layer on the zygotes;
    other loopback ports and egress stay open (a sandbox's own server works)."""
    st = svc.executor_status()["isolation"]
    net = st.get("net_layer") or {}
    if not net.get("applied"):
        pytest.skip(f"no Landlock network layer: {net}")
    deny = [int(p) for p in st["deny_ports"].split(",") if p]
    assert deny, st
    r = run(svc, f"""
        import socket, threading
        for port in {deny!r}:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=5).close()
                print("REACHED", port)
            except OSError as e:
                print("denied", port, e.errno)
        srv = socket.socket(); srv.bind(("127.0.0.1", 0)); srv.listen(1)
        port = srv.getsockname()[1]
        c = socket.create_connection(("127.0.0.1", port), timeout=5)
        conn, _ = srv.accept(); c.sendall(b"ping"); print("own server", conn.recv(4).decode())
    """)
    assert r["exit_code"] == 0, r
    assert "REACHED" not in r["stdout"] and r["stdout"].count("denied") == len(deny), r["stdout"]
    assert "own server ping" in r["stdout"]


def test_default_network_policy_refuses_the_service_ports(tmp_path):
    """The default sandbox network policy (config.sandbox_network =
    "egress:80,443"): a sandbox's own Landlock layer allows TCP connect()
    to the web ports only, so the node's gRPC / HTTP listeners (and any
    other loopback server) refuse it with EACCES, while a connect to port
    80 gets past Landlock (ECONNREFUSED: nothing listens there)."""
    from bee_code_interpreter_fs_amd.runtime import jail

    if jail.probe().get("landlock_abi", 0) < 4:
        pytest.skip("kernel without Landlock network rules")
    s = InProcess(str(tmp_path), sandbox_net_layer=False, sandbox_network="egress:80,443")
    try:
        gport = int(s.h.config.grpc_listen_addr.rpartition(":")[2])
        hport = int(s.h.config.http_listen_addr.rpartition(":")[2])
        r = run(s, f"""
            import errno, socket
            for port in ({gport}, {hport}, 80):
                try:
                    socket.create_connection(("127.0.0.1", port), timeout=5).close()
                    print(port, "REACHED")
                except OSError as e:
                    print(port, errno.errorcode.get(e.errno, e.errno))
        """)
        assert r["exit_code"] == 0, r
        assert r["stdout"].split("\n")[:3] == [f"{gport} EACCES", f"{hport} EACCES", "80 ECONNREFUSED"], r["stdout"]
    finally:
        s.stop()


APPLY_PROBE = """
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
from bee_code_interpreter_fs_amd.runtime import _jail
opts = {"own_rw": [os.getcwd()], "landlock": True, "seccomp": False}
if sys.argv[2] == "net":
    opts["net_connect_ports"] = [80, 443]
t = time.perf_counter()
st = _jail.apply(opts)
print(json.dumps({"ms": (time.perf_counter() - t) * 1e3, "net": st.get("net_connect_restricted")}))
"""


def test_network_policy_costs_no_measurable_time_per_sandbox(tmp_path):
    """The connect allow-list is a few rules in the sandbox's own layer:
    applying the jail with it takes no longer than without (the opt-in
    deny-list layer on the zygote costs ~13 ms per sandbox)."""
    from bee_code_interpreter_fs_amd.runtime import jail

    if jail.probe().get("landlock_abi", 0) < 4:
        pytest.skip("kernel without Landlock network rules")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def once(kind):
        p = subprocess.run([sys.executable, "-c", APPLY_PROBE, root, kind], cwd=str(tmp_path), capture_output=True,
                           text=True, timeout=60)
        assert p.returncode == 0, p.stderr
        return json.loads(p.stdout.strip().splitlines()[-1])

    net = [once("net") for _ in range(5)]
    plain = [once("plain") for _ in range(5)]
    assert all(x["net"] for x in net) and not any(x["net"] for x in plain)
    med = lambda xs: sorted(x["ms"] for x in xs)[len(xs) // 2]  # noqa: E731
    assert med(net) < med(plain) + 0.1, (net, plain)  # < 0.1 ms more per sandbox


def test_uid_mode_refuses_api_calls_from_sandboxes():
    """UID mode, default network policy ("open", no Landlock TCP layer): a
    sandbox reaches the service's ports, but the front-ends look up the peer
    socket's owner (services/peer_guard.py) and refuse a sandbox UID --
    PERMISSION_DENIED over gRPC, 403 over HTTP -- while /health and callers
    outside the sandboxes are served."""
    if os.geteuid() != 0:
        pytest.skip("per-sandbox UIDs need a root service")
    s = UidService(sandbox_net_layer=False, sandbox_network="open")
    try:
        host, _, gport = s.grpc_target.rpartition(":")
        hurl = str(s.http.base_url).rstrip("/")
        r = run(s, f"""
            import json, urllib.request, urllib.error
            for path in ("/v1/status", "/health"):
                try:
                    print(path, urllib.request.urlopen("{hurl}" + path, timeout=10).status)
                except urllib.error.HTTPError as e:
                    print(path, e.code, json.loads(e.read())["detail"][:40])
            req = urllib.request.Request("{hurl}/v1/execute", data=json.dumps({{"source_code": "print(1)"}}).encode(),
                                         headers={{"content-type": "application/json"}})
            try:
                print("execute", urllib.request.urlopen(req, timeout=30).status)
            except urllib.error.HTTPError as e:
                print("execute", e.code)
            import grpc
            ch = grpc.insecure_channel("{host}:{gport}")
            try:
                ch.unary_unary("/code_interpreter.v1.CodeInterpreterService/Execute")(b"", timeout=30)
                print("grpc OK")
            except grpc.RpcError as e:
                print("grpc", e.code().name)
        """)
        assert r["exit_code"] == 0, r
        out = r["stdout"].splitlines()
        assert out[0].startswith("/v1/status 403 calls from sandboxes"), out
        assert out[1:] == ["/health 200", "execute 403", "grpc PERMISSION_DENIED"], out
        # the test process (root, not a sandbox UID) is served as before
        assert s.http.get("/v1/status").status_code == 200
    finally:
        s.stop()


def test_unprivileged_mode_refuses_api_calls_from_sandboxes(tmp_path):
    """Without per-sandbox UIDs (the unprivileged service the MI355X pool
    runs: sandboxes share the service's UID) and under the default "open"
    network policy, a sandbox that calls the service's own API is refused --
    PERMISSION_DENIED over gRPC, 403 over HTTP: the front-ends ask the
    executors which running sandbox holds the peer socket
    (services/peer_guard.py, csrc/executor/sandbox_peers.cpp).  /health and
    the test process itself (same UID, not a sandbox) are served."""
    s = InProcess(str(tmp_path), sandbox_net_layer=False, sandbox_network="open", sandbox_uid_base=0)
    try:
        host, _, gport = s.grpc_target.rpartition(":")
        hurl = str(s.http.base_url).rstrip("/")
        r = run(s, f"""
            import json, urllib.request, urllib.error
            for path in ("/v1/status", "/health"):
                try:
                    print(path, urllib.request.urlopen("{hurl}" + path, timeout=10).status)
                except urllib.error.HTTPError as e:
                    print(path, e.code, json.loads(e.read())["detail"][:40])
            import grpc
            ch = grpc.insecure_channel("{host}:{gport}")
            try:
                ch.unary_unary("/code_interpreter.v1.CodeInterpreterService/Execute")(b"", timeout=30)
                print("grpc OK")
            except grpc.RpcError as e:
                print("grpc", e.code().name)
        """)
        assert r["exit_code"] == 0, r
        out = r["stdout"].splitlines()
        assert out[0].startswith("/v1/status 403 calls from sandboxes"), out
        assert out[1:] == ["/health 200", "grpc PERMISSION_DENIED"], out
        assert s.executor_status()["isolation"].get("uid_mode") in (False, None)
        # the test process (the service's own UID, no sandbox) is served, and
        # its connection's verdict is cached: later calls ask no daemon
        g = s.h.ctx.peer_guard
        assert s.http.get("/v1/status").status_code == 200
        n = g.daemon_lookups
        for _ in range(5):
            assert s.http.get("/v1/status").status_code == 200
        assert g.daemon_lookups == n
    finally:
        s.stop()
