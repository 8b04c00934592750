"""Per-sandbox resource containment, end to end on CPU.

The reference runs every execution in its own pod, and the pod's cgroup
bounds the memory, CPU and process count of everything in it
(``executor_container_resources``, `src/code_interpreter/config.py:67-68`,
applied at `services/kubernetes_code_executor.py:246`).  Here sandboxes are
forked on one node, and the executor bounds each sandbox's whole process
tree itself (csrc/executor/procmon.*; the sandbox leader is the tree's child
subreaper, so double-forked or setsid'd processes stay in it).  The limits
come from the same ``limits.memory`` / ``limits.cpu`` keys.

Each test runs in both isolation modes: ``jailed`` (Landlock + seccomp, the
sandboxes keep the service's UID -- what the unprivileged GPU box gets; as
root here RLIMIT_NPROC binds nothing, so only the monitor does) and ``uid``
(root service, a UID per sandbox).
"""

from __future__ import annotations

import os
import statistics
import threading
import time

import pytest

from .harness import wait_for
from .test_isolation_cpu import InProcess, UidService, _jail_built, run

pytestmark = pytest.mark.skipif(not _jail_built(), reason="native jail not built or Landlock ABI < 6")

LIMITS = {"limits": {"memory": "16Gi", "cpu": "1"}}
TASKS = 256


@pytest.fixture(scope="module", params=["jailed", "uid"])
def svc(request, tmp_path_factory):
    kw = dict(executor_container_resources=LIMITS, sandbox_memory_bytes=6 * 1024**3, sandbox_max_processes=TASKS)
    if request.param == "uid":
        if os.geteuid() != 0:
            pytest.skip("per-sandbox UIDs need a root service")
        s = UidService(**kw)
    else:
        s = InProcess(str(tmp_path_factory.mktemp("contain")), **kw)
    s.mode = request.param
    yield s
    s.stop()


def _tree_alive(leader: int) -> int:
    """Processes still in the sandbox leader's session or process group."""
    n = 0
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            with open(f"/proc/{pid}/stat", "rb") as fh:
                f = fh.read().rsplit(b")", 1)[1].split()
        except OSError:
            continue
        if f[0] in (b"Z", b"X"):
            continue
        if int(f[2]) == leader or int(f[3]) == leader:
            n += 1
    return n


def _alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat", "rb") as fh:
            return fh.read().rsplit(b")", 1)[1].split()[0] not in (b"Z", b"X")
    except OSError:
        return False


def test_status_reports_containment(svc):
    con = svc.executor_status()["containment"]
    assert con["memory_bytes"] == 16 * 1024**3 and con["cpus"] == 1.0 and con["tasks"] == TASKS, con
    assert con["mechanism"] == "procmon"


def test_memory_budget_covers_the_whole_tree(svc):
    """20 children of 3 GB each -- every one escaped its parent (setsid +
    double fork), as a daemonised helper would -- against a 16 GiB budget:
    the sandbox is killed as a whole once the tree holds more than that."""
    t0 = time.time()
    r = run(svc, """
        import os, time
        print(os.getpid(), flush=True)
        for i in range(20):
            if os.fork() == 0:
                os.setsid()
                if os.fork() == 0:
                    b = bytearray(b"\\x01") * (3 * 1024**3)  # every page written
                    time.sleep(120)
                os._exit(0)
        time.sleep(60)
        print("SURVIVED")
    """, timeout=120)
    took = time.time() - t0
    assert r["exit_code"] == -1, r
    assert "memory limit exceeded" in r["stderr"], r["stderr"][-500:]
    assert "SURVIVED" not in r["stdout"] and took < 50, (took, r)
    leader = int(r["stdout"].split()[0])
    assert wait_for(lambda: _tree_alive(leader) == 0, 10), _tree_alive(leader)
    assert run(svc, "print(6 * 7)")["stdout"] == "42\n"
    assert svc.executor_status()["containment"]["memory_kills"] >= 1


def test_fork_bomb_is_contained_in_every_mode(svc):
    """2^11 processes (bounded, so a broken monitor cannot take the test box
    down) against a 256-task budget.  Without root (``jailed``; as root here
    RLIMIT_NPROC binds nothing either) the executor's monitor kills the tree;
    in UID mode RLIMIT_NPROC of the sandbox UID refuses the forks first.
    Either way nothing of the tree outlives the sandbox."""
    t0 = time.time()
    r = run(svc, """
        import os, time
        print(os.getpid(), flush=True)
        for _ in range(11):
            try:
                os.fork()
            except OSError:
                break
        time.sleep(5)
        if os.getpgrp() == os.getpid():
            print("SURVIVED")
    """, timeout=90)
    if svc.mode == "jailed":
        assert r["exit_code"] == -1 and "process limit exceeded" in r["stderr"], r
        assert "SURVIVED" not in r["stdout"], r
    else:
        assert r["exit_code"] == 0 or "process limit exceeded" in r["stderr"], r
    assert time.time() - t0 < 60
    leader = int(r["stdout"].split()[0])
    assert wait_for(lambda: _tree_alive(leader) == 0, 15), _tree_alive(leader)
    assert run(svc, "print(6 * 7)")["stdout"] == "42\n"


NEIGHBOR = """
import time
t = time.perf_counter()
s = 0
for i in range(3_000_000):
    s += i
print(round(time.perf_counter() - t, 4))
"""

HOG = """
import os, time
for _ in range(31):
    if os.fork() == 0:
        while True:
            pass
t0, c0 = time.time(), time.process_time()
while time.time() - t0 < 10:
    pass
print("hog main cpu share", round((time.process_time() - c0) / (time.time() - t0), 3))
"""


def test_cpu_hog_is_throttled_to_its_share(svc):
    """A 32-process CPU hog with limits.cpu = 1 gets about one core: its own
    main process sees ~1/32 of a core (8/32 unthrottled on this 8-CPU box),
    and a neighbour sandbox's run time stays within 2x of its time alone."""

    def neighbor_p50(n=7):
        return statistics.median(float(run(svc, NEIGHBOR)["stdout"]) for _ in range(n))

    alone = neighbor_p50()
    hog = {}
    th = threading.Thread(target=lambda: hog.setdefault("r", run(svc, HOG, timeout=60)))
    before = svc.executor_status()["containment"]["cpu_throttles"]
    th.start()
    try:
        time.sleep(1.0)
        busy = neighbor_p50()
    finally:
        th.join(90)
    r = hog["r"]
    assert r["exit_code"] == 0, r
    share = float(r["stdout"].split()[-1])
    assert share < 0.12, r["stdout"]
    assert busy < 2 * alone, (alone, busy)
    assert svc.executor_status()["containment"]["cpu_throttles"] > before


def test_namespace_clones_and_subreaper_are_refused(svc):
    r = run(svc, """
        import ctypes, os, threading
        libc = ctypes.CDLL(None, use_errno=True)
        libc.syscall.restype = ctypes.c_long
        SYS_clone, SYS_clone3 = 56, 435
        for flag in (0x10000000, 0x40000000, 0x00020000, 0x20000000):  # NEWUSER NEWNET NEWNS NEWPID
            rc = libc.syscall(SYS_clone, flag | 17, 0, 0, 0, 0)
            if rc == 0:
                os._exit(0)
            print("clone", hex(flag), rc, ctypes.get_errno())
        print("clone3", libc.syscall(SYS_clone3, 0, 0), ctypes.get_errno())
        print("subreaper_off", libc.prctl(36, 0, 0, 0, 0), ctypes.get_errno())
        v = ctypes.c_int()
        libc.prctl(37, ctypes.byref(v), 0, 0, 0)
        print("is_subreaper", v.value)
        pid = os.fork()
        if pid == 0:
            os._exit(3)
        print("fork", os.waitpid(pid, 0)[1] >> 8)
        t = threading.Thread(target=lambda: print("thread ok"))
        t.start(); t.join()
    """)
    assert r["exit_code"] == 0, r
    out = r["stdout"]
    assert out.count(" -1 1\n") == 4 + 1, out  # four namespace clones + subreaper_off: EPERM
    assert "clone3 -1 38" in out, out           # ENOSYS: libc falls back to clone
    assert "is_subreaper 1" in out and "fork 3" in out and "thread ok" in out, out


def test_escaped_daemon_dies_with_its_sandbox(svc):
    token = f"/dev/shm/bee-esc-{os.getpid()}-{svc.mode}"
    r = run(svc, f"""
        import os, time
        if os.fork() == 0:
            os.setsid()
            if os.fork() == 0:
                open({token!r}, "w").write(str(os.getpid()))
                time.sleep(120)
            os._exit(0)
        for _ in range(200):
            if os.path.exists({token!r}):
                break
            time.sleep(0.01)
        time.sleep(0.05)
        print(open({token!r}).read(), os.getpid())
    """)
    try:
        os.unlink(token)
    except OSError:
        pass
    assert r["exit_code"] == 0, r
    daemon, leader = (int(x) for x in r["stdout"].split())
    assert wait_for(lambda: not _alive(daemon), 5)
    assert _tree_alive(leader) == 0


# ---- cgroup v2 leaves ------------------------------------------------------------------


def test_cgroup_leaves_are_off_without_a_delegated_subtree(svc):
    """Neither this container (cgroup v1) nor the GPU box (a root-owned
    cgroup v2 directory, service as an unprivileged user) delegates a
    subtree: the monitor contains sandboxes and status says why."""
    con = svc.executor_status()["containment"]
    cg = con["cgroup2"]
    if cg["enabled"]:
        pytest.skip(f"this node delegates a cgroup v2 subtree ({cg['base']})")
    assert con["mechanism"] == "procmon" and cg["reason"], con


def test_cgroup_leaf_per_sandbox(tmp_path):
    """With a delegated subtree (here a plain directory standing in for it:
    --cgroup=fake), every sandbox gets its own leaf with the pod's bounds --
    memory.max, swap off, OOM kills the whole group, pids.max, cpu.max -- and
    joins it before its job runs; the leaf is removed afterwards."""
    root = tmp_path / "cg"
    root.mkdir()
    (root / "cgroup.controllers").write_text("cpuset cpu io memory pids\n")
    (root / "cgroup.subtree_control").write_text("")
    s = InProcess(str(tmp_path / "svc"), executor_container_resources={"limits": {"memory": "3Gi", "cpu": "1.5"}},
                  sandbox_max_processes=200, sandbox_cgroup="fake", sandbox_cgroup_root=str(root))
    try:
        con = s.executor_status()["containment"]
        assert con["mechanism"] == "cgroup2+procmon" and con["cgroup2"]["enabled"], con
        assert con["cgroup2"]["base"] == str(root)
        seen = {}
        done = threading.Event()

        def watch():
            while not done.is_set():
                for leaf in root.iterdir():
                    if leaf.is_dir() and leaf.name.startswith("bee-") and (leaf / "cgroup.procs").exists():
                        try:
                            snap = {f.name: f.read_text() for f in leaf.iterdir()}
                        except OSError:
                            continue
                        # keep the last snapshot taken while the sandbox was
                        # in it (a read racing the leaf's set-up or teardown
                        # must not replace it)
                        if snap.get("cgroup.procs", "").strip():
                            seen[leaf.name] = snap
                time.sleep(0.01)

        t = threading.Thread(target=watch)
        t.start()
        try:
            r = run(s, "import os, time; print(os.getpid()); time.sleep(1.0)")
        finally:
            done.set()
            t.join()
        assert r["exit_code"] == 0, r
        pid = r["stdout"].split()[0]
        files = [f for f in seen.values() if f.get("cgroup.procs", "").strip() == pid]
        assert files, seen
        f = files[0]
        assert f["memory.max"] == str(3 * 1024**3) and f["memory.swap.max"] == "0" and f["memory.oom.group"] == "1", f
        assert f["pids.max"] == "200" and f["cpu.max"] == "150000 100000", f
        assert "memory" in (root / "cgroup.subtree_control").read_text()
        # removed once the sandbox is gone
        assert wait_for(lambda: not any(p.name.startswith("bee-") for p in root.iterdir()), timeout=15), list(root.iterdir())
        assert s.executor_status()["containment"]["cgroup2"]["leaves"] >= 1
    finally:
        s.stop()
