"""Single-use sandbox worker (runs in a child forked from the zygote).

Lifecycle (driven by the native executor, csrc/executor/sandbox.cpp):

1. ``setsid`` — the worker leads its own session and process group, so the
   executor can kill everything the user code started with one ``killpg``;
2. apply the sandbox environment (GPU pin via ``HIP_VISIBLE_DEVICES``, dirs,
   HBM quota) — HIP is still uninitialised in the zygote, so this is legal;
3. connect to the executor, say ``hello``;
4. warm up: ``beekern.init()`` creates the HIP context on the pinned GPU and
   loads the kernel code object (the 0.1-0.5 s the MI355X probe measured),
   then ``ready`` — all of this while the sandbox waits in the pool;
5. block for exactly one ``run``; execute the script with python semantics
   (compiled as ``__main__``), stdout/stderr to files, then exit.

The reference ran every script through ``xonsh`` in a fresh interpreter
(`executor/server.rs:197-206`); python semantics here are what its own TODO
asks for (~80 ms saved) and what the examples need.
"""

from __future__ import annotations

import binascii  # precompiled payloads (load_precompiled): imported pre-fork
import builtins
import ctypes
import io
import json
import marshal
import os
import resource
import socket
import sys
import time
import traceback
import types
from typing import Optional

SANDBOX_SITE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sandbox_site")
_STAMPS: dict = {}  # phase timestamps reported to the executor


class _Chan:
    """The sandbox's line-JSON channel to the executor, on a raw descriptor
    (no socket object: its class machinery alone cost ~120 copy-on-write
    faults per sandbox)."""

    __slots__ = ("fd", "buf")

    def __init__(self, fd: int) -> None:
        self.fd = fd
        self.buf = b""

    def send(self, data: bytes) -> None:
        view = memoryview(data)
        while view:
            view = view[os.write(self.fd, view):]

    def recv_json(self) -> Optional[dict]:
        while b"\n" not in self.buf:
            chunk = os.read(self.fd, 65536)
            if not chunk:
                return None
            self.buf += chunk
        line, self.buf = self.buf.split(b"\n", 1)
        return json.loads(line)


def _json_str(s: str) -> str:
    return json.dumps(s) if s else '""'


_OUT_FDS: dict = {}  # stdout / stderr / timing.json, opened before the jail
_REDIRECTED: list = []  # [stdout path, stderr path] once fds 1 / 2 point at the run's files


def _open_outputs(meta_dir: str) -> None:
    """Open the run's output files while the sandbox still runs as the
    executor's user: the meta directory is the executor's (0700), so after
    the jail the sandbox can write these descriptors but cannot reach (or
    swap) the files themselves."""
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_NOFOLLOW | os.O_CLOEXEC
    for name in ("stdout", "stderr", "timing.json"):
        _OUT_FDS[name] = os.open(os.path.join(meta_dir, name), flags, 0o600)


_STDIO: Optional[tuple] = None  # (stdin, stdout, stderr) text layers over fds 0/1/2, built by the zygote


def prepare_stdio() -> None:
    """Zygote, before forking: the text layers a `python script.py` run has
    over fds 0/1/2, built once (closefd=False, empty buffers at the fork) and
    installed as the zygote's own sys.std*, so a sandbox only points the
    descriptors at its run's files.  Building them per sandbox -- three
    FileIO / BufferedWriter / TextIOWrapper stacks, codec lookups, and the
    deallocation of the zygote's layers they replaced -- measured 0.2 ms and
    ~110 copy-on-write faults of every sandbox's CPU on MI355X.  Built while
    fds 0/1/2 point at /dev/null, so the layers see what a run's regular
    files look like (seekable, position 0)."""
    global _STDIO
    for stream in (sys.stdout, sys.stderr):
        try:
            stream.flush()
        except Exception:
            pass
    null_fd = os.open(os.devnull, os.O_RDWR)
    saved = [os.dup(fd) for fd in (0, 1, 2)]
    try:
        for fd in (0, 1, 2):
            os.dup2(null_fd, fd)
        stdin = io.TextIOWrapper(io.FileIO(0, "r", closefd=False), encoding="utf-8")
        stdout = io.TextIOWrapper(
            io.BufferedWriter(io.FileIO(1, "w", closefd=False)), encoding="utf-8", errors="backslashreplace"
        )
        stderr = io.TextIOWrapper(
            io.BufferedWriter(io.FileIO(2, "w", closefd=False)),
            encoding="utf-8",
            errors="backslashreplace",
            line_buffering=True,
        )
    finally:
        for fd, keep in zip((0, 1, 2), saved):
            os.dup2(keep, fd)
            os.close(keep)
        os.close(null_fd)
    _STDIO = (stdin, stdout, stderr)
    sys.stdin, sys.stdout, sys.stderr = _STDIO
    sys.__stdin__, sys.__stdout__, sys.__stderr__ = _STDIO


def _redirect_stdio(stdout_path: str, stderr_path: str) -> None:
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC
    out_fd = _OUT_FDS.pop("stdout", None)
    err_fd = _OUT_FDS.pop("stderr", None)
    _REDIRECTED[:] = [stdout_path, stderr_path]
    if out_fd is None:
        out_fd = os.open(stdout_path, flags, 0o600)
    if err_fd is None:
        err_fd = os.open(stderr_path, flags, 0o600)
    null_fd = os.open(os.devnull, os.O_RDONLY)
    os.dup2(null_fd, 0)
    os.dup2(out_fd, 1)
    os.dup2(err_fd, 2)
    for fd in (out_fd, err_fd, null_fd):
        os.close(fd)
    if _STDIO is not None and not _STDIO[1].closed and not _STDIO[2].closed:
        # the zygote's layers (prepare_stdio): nothing buffered, now over the run's files
        for stream in _STDIO[1:]:
            stream.flush()
        sys.stdin, sys.stdout, sys.stderr = _STDIO
        sys.__stdin__, sys.__stdout__, sys.__stderr__ = _STDIO
        return
    # fresh text layers like a normal `python script.py` writing to files
    sys.stdin = io.TextIOWrapper(io.FileIO(0, "r", closefd=False), encoding="utf-8")
    sys.stdout = io.TextIOWrapper(
        io.BufferedWriter(io.FileIO(1, "w", closefd=False)), encoding="utf-8", errors="backslashreplace"
    )
    sys.stderr = io.TextIOWrapper(
        io.BufferedWriter(io.FileIO(2, "w", closefd=False)),
        encoding="utf-8",
        errors="backslashreplace",
        line_buffering=True,
    )
    sys.__stdout__, sys.__stderr__, sys.__stdin__ = sys.stdout, sys.stderr, sys.stdin


def _print_user_traceback(exc: BaseException, script: str) -> None:
    """Traceback as `python script.py` shows it: drop runner frames."""
    tb = exc.__traceback__
    while tb is not None and os.path.abspath(tb.tb_frame.f_code.co_filename) != os.path.abspath(script):
        tb = tb.tb_next
    te = traceback.TracebackException(type(exc), exc, tb if tb is not None else exc.__traceback__)
    sys.stderr.write("".join(te.format()))


def _resolve_fsmap():
    try:
        fn = ctypes.CDLL(None).bee_fsmap_set
        fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        fn.restype = None
        return fn
    except (AttributeError, OSError):
        return None


_FSMAP_SET = _resolve_fsmap()  # resolved once in the zygote (the shim is preloaded there)


def _resolve_fsmap_tmp():
    try:
        fn = ctypes.CDLL(None).bee_fsmap_set_tmp
        fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        fn.restype = None
        return fn
    except (AttributeError, OSError):
        return None


_FSMAP_SET_TMP = _resolve_fsmap_tmp()


def _logical_view(workspace: str, runtime_packages: str):
    """Give this sandbox its own ``/workspace`` and ``/runtime-packages``
    (the reference pod's layout, executor/server.rs:68-74) through the
    preloaded libc path shim (csrc/fsmap/fsmap.cpp).  Returns the paths as
    the user's code sees them; unchanged when the shim is not loaded (pod
    mode, where those directories are real)."""
    if _FSMAP_SET is None or workspace == "/workspace":
        return workspace, runtime_packages
    _FSMAP_SET(os.fsencode(workspace), os.fsencode(runtime_packages or ""))
    tmp = os.environ.get("TMPDIR", "")
    if _FSMAP_SET_TMP is not None and tmp and os.environ.get("BEE_JAIL") == "1":
        # jailed: the host's /tmp is outside the sandbox's view; give it its
        # own, except for the host trees below /tmp that its view includes
        from . import jail

        keep = jail.visible_under("/tmp")
        if os.environ.get("BEE_JAIL_SHARED"):  # gang ranks: rank 0's tmp (the script)
            keep.append(os.path.realpath(os.environ["BEE_JAIL_SHARED"]))
        _FSMAP_SET_TMP(os.fsencode(tmp), os.fsencode(":".join(keep)))
    os.environ["PWD"] = "/workspace"
    return "/workspace", ("/runtime-packages" if runtime_packages else "")


def _to_logical(path: str, real_root: str, logical_root: str) -> str:
    # the executor hands out absolute, normalised sandbox paths
    real_root = real_root.rstrip(os.sep)
    if path == real_root or path.startswith(real_root + os.sep):
        return logical_root + path[len(real_root):]
    return path


def _apply_limits() -> None:
    resource.setrlimit(resource.RLIMIT_CORE, (0, 0))
    fsize = os.environ.get("BEE_RLIMIT_FSIZE")
    if fsize:
        resource.setrlimit(resource.RLIMIT_FSIZE, (int(fsize), int(fsize)))


def warm_gpu() -> Optional[str]:
    """Direct sandboxes: create the HIP context and load the kernel library.
    Light sandboxes: open the session with the executor's kernel broker.
    Returns an error string (the sandbox stays usable for CPU code)."""
    try:
        from bee_code_interpreter_fs_amd import ops

        # BEE_BROKER_LAZY=1: a light/minimal sandbox opens its broker session
        # on first use instead of while pooled.  BEE_DEVICE: the device of a
        # warm gang rank (rank r of a gang holds device r of its visible list)
        device = int(os.environ.get("BEE_DEVICE", "0") or 0)
        ops.init(device, lazy=os.environ.get("BEE_BROKER_LAZY") == "1")
        quota = int(os.environ.get("BEE_HBM_QUOTA_BYTES", "0") or 0)
        if quota > 0 and ops.driver_name() == "native":
            ops.set_quota(quota)
        if os.environ.get("BEE_WARM_TORCH") == "1" and "torch" in sys.modules:
            # torch's own CUDA state too (lazy init, the caching allocator's
            # first block): a gang rank's `torch.cuda.set_device(LOCAL_RANK)`
            # and first tensor then cost nothing on the request path
            torch = sys.modules["torch"]
            torch.cuda.set_device(device)
            torch.zeros(1, device="cuda").add_(1)
            torch.cuda.synchronize()
        return None
    except Exception as e:  # keep the sandbox usable for CPU code
        return f"{type(e).__name__}: {e}"


from importlib.util import MAGIC_NUMBER as _MAGIC  # noqa: E402 - the interpreter's bytecode magic, pre-fork


def load_precompiled(blob: str, path: str):
    """(code object, needs the shell runtime) from the front-end's
    precompiled payload (scheduler/local_gpu_pool.py precompiled), with every
    code object's file name set to ``path`` as compile(source, path) would
    have; None when the blob is not for this interpreter or does not decode
    (the worker then compiles the source itself)."""
    try:
        raw = binascii.a2b_base64(blob)
    except (binascii.Error, ValueError):
        return None
    magic = _MAGIC
    if raw[: len(magic)] != magic or raw[len(magic): len(magic) + 1] not in (b"P", b"X"):
        return None
    try:
        code = marshal.loads(raw[len(magic) + 1:])
    except (EOFError, ValueError, TypeError):
        return None
    if not isinstance(code, types.CodeType):
        return None

    def rename(c):
        consts = tuple(rename(k) if isinstance(k, types.CodeType) else k for k in c.co_consts)
        return c.replace(co_filename=path, co_consts=consts)

    return rename(code), raw[len(magic): len(magic) + 1] == b"X"


def _run_main(path: str, lowered: Optional[str] = None, code=None, shell: bool = False,
              raw: Optional[bytes] = None) -> None:
    """`python path` semantics (what runpy.run_path does for a plain file,
    minus its zip/directory probing): compile, bind a fresh ``__main__``
    module, execute.  ``lowered``: the payload with its xonsh shell lines
    lowered to Python (runtime/xsh.py), compiled under the same file name so
    tracebacks point at the user's lines.  ``raw``: the file's bytes when the
    caller already read them (compile() honours a coding cookie in bytes, as
    for the file).  The module is left alive -- the
    process ends with os._exit, and the broker releases device memory on
    disconnect -- so no teardown work lands on the request path."""
    if code is None:
        if lowered is None and raw is not None:
            source = raw
        elif lowered is None:
            with io.open_code(path) as fh:
                source = fh.read()
        else:
            source = lowered
        code = compile(source, path, "exec", dont_inherit=True)
        shell = lowered is not None
    mod = types.ModuleType("__main__")
    mod.__dict__.update({"__file__": path, "__cached__": None, "__loader__": None, "__package__": None,
                         "__spec__": None, "__builtins__": builtins})
    if shell:
        from . import xsh

        mod.__dict__[xsh.RUNTIME_NAME] = xsh.Runtime()
    sys.modules["__main__"] = mod
    try:
        exec(code, mod.__dict__)
    finally:
        _STAMPS["exec_end"] = time.monotonic() * 1e3
        _KEEP.append(mod)


_KEEP: list = []


_PATHS_FOR: list = []  # the runtime-packages view _prepare_paths ran for
_NUMPY_OFFLOAD: list = []  # non-empty: this run asked for the numpy offload


def _prepare_paths(runtime_packages: str) -> None:
    """sys.path and PYTHONPATH of a `python script.py` run with the
    runtime-packages tree importable (what the reference's image set up);
    done while pooled, the script's own directory is added at run time."""
    sys.path[:] = [p for p in sys.path if p not in ("", ".")]
    if runtime_packages and runtime_packages not in sys.path:
        sys.path.insert(0, runtime_packages)
    if SANDBOX_SITE not in sys.path:
        sys.path.append(SANDBOX_SITE)
    pp = os.environ.get("PYTHONPATH", "")
    os.environ["PYTHONPATH"] = os.pathsep.join(p for p in (runtime_packages, SANDBOX_SITE, pp) if p)
    _PATHS_FOR[:] = [runtime_packages]


def run_script(script: str, argv, workspace: str, runtime_packages: str, precompiled: Optional[str] = None) -> int:
    sys.argv = [script, *argv]
    script_dir = os.path.dirname(os.path.abspath(script))
    if _PATHS_FOR != [runtime_packages]:
        _prepare_paths(runtime_packages)
    sys.path.insert(0, script_dir)
    from . import sandbox_patches

    sandbox_patches.install()
    if _NUMPY_OFFLOAD:
        # large numpy.random draws live on the GPU and numpy calls on them
        # dispatch to the kernels (ops/numpy_offload.py)
        from bee_code_interpreter_fs_amd.ops import numpy_offload

        numpy_offload.install()
    lowered = None
    raw = None
    pre = load_precompiled(precompiled, script) if precompiled else None
    # the dependency guesser needs the source only with a wheelhouse to install from
    guess = bool(os.environ.get("BEE_WHEELHOUSE"))
    try:
        if pre is None or guess:
            # read once: the lowering, the guesser and the compile share it
            with io.open_code(script) as fh:
                raw = fh.read()
            source = raw.decode("utf-8", errors="replace")
            from . import xsh
            from .deps import install_missing

            # xonsh-style shell lines (the reference ran every payload through
            # xonsh): lowered to Python here, plain Python passes untouched --
            # unless the front-end already compiled the payload (lowering included)
            if pre is None:
                lowered = xsh.lower_payload(source)
            if guess:
                install_missing(lowered or source, runtime_packages)
    except OSError:
        pass
    code = 0
    _STAMPS["script_start"] = time.monotonic() * 1e3
    try:
        if pre is not None:
            _run_main(script, code=pre[0], shell=pre[1])
        else:
            _run_main(script, lowered, raw=raw)
    except SystemExit as e:
        if e.code is None:
            code = 0
        elif isinstance(e.code, int):
            code = e.code
        else:
            sys.stderr.write(f"{e.code}\n")
            code = 1
    except KeyboardInterrupt:
        code = 130
    except BaseException as e:  # noqa: BLE001 - report like the interpreter does
        _print_user_traceback(e, script)
        code = 1
    return code


ZYGOTE_MODULES: frozenset = frozenset()  # set by the zygote before it forks


def _finish(code: int, timing_path: Optional[str] = None, chan: Optional[_Chan] = None) -> None:
    _STAMPS["script_end"] = time.monotonic() * 1e3
    _cow_report()
    if os.environ.get("BEE_DEBUG_NEW_MODULES") == "1" and ZYGOTE_MODULES:
        # diagnostics: modules this sandbox imported that its zygote had not
        # (each one is paid for on every execution)
        sys.stderr.write("NEW_MODULES " + " ".join(sorted(set(sys.modules) - ZYGOTE_MODULES)) + "\n")
        t0 = _STAMPS.get("recv", 0)
        sys.stderr.write("STAMPS " + json.dumps({k: (v if k.startswith(("cpu_", "flt_", "minflt", "cow_")) else round(v - t0, 3))
                                                 for k, v in _STAMPS.items()}) + "\n")
    try:
        import atexit

        atexit._run_exitfuncs()  # only the user's: the zygote cleared its own
        if "logging" in sys.modules:
            sys.modules["logging"].shutdown()
    except BaseException:
        pass
    for stream in (sys.stdout, sys.stderr):
        try:
            stream.flush()
        except Exception:
            pass
    _STAMPS["exit"] = time.monotonic() * 1e3
    try:
        ru = resource.getrusage(resource.RUSAGE_SELF)
        _STAMPS["cpu_ms"] = (ru.ru_utime + ru.ru_stime) * 1e3
        _STAMPS["minflt"] = ru.ru_minflt
    except Exception:
        pass
    status = code & 0xFF if code >= 0 else 1
    tfd = _OUT_FDS.pop("timing.json", None)
    if tfd is not None or timing_path:
        try:  # CLOCK_MONOTONIC ms, the executor's clock too
            with (os.fdopen(tfd, "w") if tfd is not None else open(timing_path, "w")) as fh:
                json.dump(_STAMPS, fh)
        except OSError:
            pass
    if chan is not None:
        # outputs are flushed: the executor can answer now and reap this
        # process (and anything it left behind) off the request path
        try:
            chan.send(b'{"op":"done","code":%d}\n' % status)
            # stay, stopped in a read, until the executor kills the tree: this
            # process is its sandbox's child subreaper, so whatever the script
            # left running (double-forked, setsid'd) is still below it when
            # the executor walks the tree to kill it (a channel EOF -- the
            # executor gone -- ends the wait)
            while os.read(chan.fd, 4096):
                pass
        except OSError:
            pass
    os._exit(status)


def _cow_mark() -> None:
    """A learner sandbox notes the zygote pages it holds before its request
    arrives: only what the request path writes is learned."""
    zl = sys.modules.get("bee_code_interpreter_fs_amd.runtime._zygote_loop")
    if zl is not None and hasattr(zl, "cow_mark"):
        try:
            zl.cow_mark()
        except Exception:
            pass


def _cow_begin(trusted: bool) -> None:
    """A learner sandbox whose job just arrived tells its zygote, before any
    user code runs, whether the job is the service's own (its set is then
    trusted; csrc/zygote/zygote_loop.cpp "Trust").  A no-op elsewhere."""
    zl = sys.modules.get("bee_code_interpreter_fs_amd.runtime._zygote_loop")
    if zl is None or not hasattr(zl, "cow_begin"):
        return
    try:
        if zl.cow_begin(trusted) is not None and _DEBUG:
            _STAMPS["cow_trusted"] = int(trusted)
    except Exception:
        pass


def _cow_report() -> None:
    """A learner sandbox tells its zygote which of the zygote's pages it
    wrote, before it reports done (csrc/zygote/zygote_loop.cpp "copy-on-write
    prefault"): later sandboxes copy them up front while pooled.  A no-op in
    every other sandbox."""
    zl = sys.modules.get("bee_code_interpreter_fs_amd.runtime._zygote_loop")
    if zl is None or not hasattr(zl, "cow_report"):
        return
    try:
        got = zl.cow_report()
        if _DEBUG:
            st = zl.cow_stats()
            _STAMPS["cow_prefault_pages"] = st["prefault_pages"]
            _STAMPS["cow_prefault_ms"] = round(st["prefault_ms"], 3)
            _STAMPS["cow_trusted_pages"] = st.get("trusted_pages", 0)  # the zygote's view at this fork
            _STAMPS["cow_rejected"] = st.get("rejected", 0)
            if got is not None:
                (_STAMPS["cow_learned_runs"], _STAMPS["cow_learned_pages"], _STAMPS["cow_entry_maps"],
                 _STAMPS["cow_scanned_pages"], _STAMPS["cow_pagemap_open"]) = got
    except Exception:
        pass


_LIGHT_WARMUP = """
import numpy as np, pandas as pd
df = pd.DataFrame({"a": np.arange(64.0), "b": np.arange(64.0)[::-1]})
df["c"] = df["a"] * 2 + df["b"]
s = df.describe().loc[["mean", "std"]].to_string()
"""


def _prefault_scientific() -> None:
    """Light sandboxes (pandas / scipy preloaded): touch the common
    DataFrame construction / arithmetic / describe / printing paths while
    pooled.  A light
    sandbox's first pandas call otherwise pays thousands of copy-on-write
    faults on the request path (the objects it touches are the zygote's)."""
    if os.environ.get("BEE_ZYGOTE_KIND") != "light" or "pandas" not in sys.modules:
        return
    if os.environ.get("BEE_LIGHT_WARMUP", "1") == "0":
        return
    try:
        exec(compile(_LIGHT_WARMUP, "<light-warmup>", "exec", dont_inherit=True), {"__name__": "__warmup__"})
    except Exception:
        pass


def _prefault() -> None:
    """Run the request path's Python machinery once while the sandbox waits
    in the pool: a freshly forked process pays a copy-on-write fault on every
    page it first writes (allocator pools, refcounts of shared objects), and
    this moves those faults off the request path."""
    try:
        doc = json.loads(json.dumps({"op": "run", "script": "/x", "argv": [], "env": {"A": "1"}}))
        code = compile("import sys\nx = [i * i for i in range(64)]\n", "<prefault>", "exec", dont_inherit=True)
        exec(code, {"__builtins__": builtins, "__name__": "__prefault__"})
        os.environ["BEE_PREFAULT_SCRATCH"] = doc["env"]["A"]
        del os.environ["BEE_PREFAULT_SCRATCH"]
        _to_logical("/a/b", "/a", "/workspace")
        io.TextIOWrapper(io.BufferedWriter(io.FileIO(os.open(os.devnull, os.O_WRONLY), "w")), encoding="utf-8").close()
        if os.environ.get("BEE_PREFAULT_TB") == "1":
            traceback.TracebackException(ValueError, ValueError("x"), None).format()
    except Exception:
        pass


def reseed_entropy_state() -> None:
    """Give this sandbox its own numpy legacy RandomState stream.

    A fresh interpreter (the reference's process per run) seeds numpy's
    global RandomState from OS entropy at import; sandboxes forked from a
    zygote would all inherit the zygote's, so every execution would draw the
    same ``np.random.rand()`` (and scipy's default ``random_state``, which is
    the same object).  The full 19968-bit MT19937 state is replaced from the
    OS in one C call: ~0.4 ms less copy-on-write work than ``seed()``'s
    SeedSequence path, and nothing that captured the object at import is
    left on the old stream."""
    npr = sys.modules.get("numpy.random")
    if npr is None:
        return
    try:
        import numpy as np

        npr.mtrand._rand.set_state(("MT19937", np.frombuffer(os.urandom(2496), dtype=np.uint32), 624))
    except Exception:  # keep the sandbox usable; the stream is then the zygote's
        pass


_DEBUG = False  # BEE_DEBUG_NEW_MODULES=1: per-phase CPU / fault stamps of the pooled phase


def _cpu_stamp_force(name: str) -> None:
    ru = resource.getrusage(resource.RUSAGE_SELF)
    _STAMPS["cpu_" + name] = round((ru.ru_utime + ru.ru_stime) * 1e3, 3)
    _STAMPS["flt_" + name] = ru.ru_minflt


def _cpu_stamp(name: str) -> None:
    if _DEBUG:
        _cpu_stamp_force(name)


def _resolve_hbm_latch():
    try:
        fn = ctypes.CDLL(None).bee_hbm_quota_latch  # the LD_PRELOADed interposer
        fn.argtypes = [ctypes.c_int64]
        fn.restype = ctypes.c_int
        return fn
    except (AttributeError, OSError):
        return None


_HBM_LATCH = _resolve_hbm_latch()


QUOTA_FD = 1013  # csrc/hbm_quota/hbm_quota.cpp kQuotaFd


def _publish_quota_memfd(quota: int) -> None:
    """The run's quota for programs this sandbox execs: a sealed memfd at a
    fixed descriptor, inherited across exec (the interposer's constructor
    latches from it -- or from an ancestor's, when a launcher closed it --
    before it would read BEE_HBM_QUOTA_BYTES, which the child's environment
    may set to anything).  Sealed: nobody rewrites the value in place."""
    import fcntl

    try:
        fd = os.memfd_create("bee-hbm-quota", os.MFD_ALLOW_SEALING)  # no CLOEXEC: exec'd programs keep it
        try:
            os.write(fd, int(quota).to_bytes(8, "little", signed=True))
            fcntl.fcntl(fd, fcntl.F_ADD_SEALS,
                        fcntl.F_SEAL_WRITE | fcntl.F_SEAL_SHRINK | fcntl.F_SEAL_GROW | fcntl.F_SEAL_SEAL)
            os.dup2(fd, QUOTA_FD, inheritable=True)
        finally:
            os.close(fd)
    except (OSError, AttributeError):
        pass  # the environment (and the executor's watchdog) still apply


def _apply_job_quota(quota: int) -> None:
    """The run's HBM quota, before user code: the interposer (direct
    sandboxes) and a native beekern context enforce it in-process, a broker
    session is charged by the daemon (the client only learns it, for early
    refusals)."""
    if _HBM_LATCH is not None:
        _HBM_LATCH(max(int(quota), 0))  # fixed for this process from here on
    if quota <= 0:
        return
    if _HBM_LATCH is not None:
        _publish_quota_memfd(quota)
    os.environ["BEE_HBM_QUOTA_BYTES"] = str(quota)
    if "bee_code_interpreter_fs_amd.ops.array" not in sys.modules:
        return
    from bee_code_interpreter_fs_amd import ops

    if not ops.is_initialized():
        return
    if ops.driver_name() == "native":
        ops.set_quota(quota)
    elif ops.driver_name() == "broker":
        # (the package exports a function named `array`: reach the module itself)
        sys.modules["bee_code_interpreter_fs_amd.ops.array"].driver().note_quota(quota)


def worker_main(spawn: dict) -> None:
    """Entry point in the forked child when the zygote did not bootstrap it
    natively (csrc/zygote/zygote_loop.cpp boot_child does these same steps
    in C); never returns."""
    global _DEBUG
    try:
        _DEBUG = os.environ.get("BEE_DEBUG_NEW_MODULES") == "1"
        _cpu_stamp("forked")
        if os.environ.get("BEE_SANDBOX_SETSID") == "0":
            os.setpgid(0, 0)  # a group of its own in the zygote's session (boot_child)
        else:
            os.setsid()
        # this sandbox's tree keeps its orphans (a double fork re-parents to
        # us, not to the zygote): the executor accounts and kills them with it
        import ctypes

        ctypes.CDLL(None, use_errno=True).prctl(36, 1, 0, 0, 0)  # PR_SET_CHILD_SUBREAPER
        env = spawn.get("env") or {}
        if env.get("BEE_CPU_AFFINITY"):  # a gang rank: its GPU's slot CPUs (boot_child does the same)
            from ..scheduler.topology import parse_cpulist

            os.sched_setaffinity(0, parse_cpulist(env["BEE_CPU_AFFINITY"]))
        os.environ.update({k: str(v) for k, v in env.items()})
        for k in spawn.get("unset") or ():  # zygote-environment entries this sandbox must not have
            os.environ.pop(k, None)
        cwd = spawn.get("cwd") or os.environ.get("BEE_WORKSPACE", ".")
        os.chdir(cwd)
        _apply_limits()
        sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        sock.connect(os.environ["BEE_WORKER_SOCK"])
        chan = _Chan(sock.detach())
        chan.send((json.dumps({"op": "hello", "id": spawn["id"], "pid": os.getpid()}) + "\n").encode())
        meta = os.environ.get("BEE_META_DIR")
        if meta:
            _open_outputs(meta)
    except BaseException:
        try:
            traceback.print_exc()
        finally:
            os._exit(70)
    _serve(cwd, chan)


def worker_main_booted(boot: tuple) -> None:
    """Entry point in the forked child after the zygote's native bootstrap:
    session, environment, cwd, rlimits, hello and output files are done;
    ``boot`` = (id, cwd, channel fd, (stdout, stderr, timing fds) | None).
    Never returns."""
    global _DEBUG
    _DEBUG = os.environ.get("BEE_DEBUG_NEW_MODULES") == "1"
    _cpu_stamp("forked")
    _, cwd, fd, outs = boot
    if outs is not None:
        _OUT_FDS["stdout"], _OUT_FDS["stderr"], _OUT_FDS["timing.json"] = outs
    _serve(cwd, _Chan(fd))


def _serve(cwd: str, chan: _Chan) -> None:
    """The pooled sandbox: jail, warm up, report ready, run the one job."""
    try:
        # the isolation boundary (runtime/jail.py): from here on this process
        # is the sandbox -- its own UID when the executor assigned one, its
        # own filesystem view, signal/ptrace scope and syscall filter
        from . import jail

        jail.apply([cwd, os.environ.get("BEE_RUNTIME_PACKAGES", ""), os.environ.get("TMPDIR", ""),
                    os.environ.get("BEE_JAIL_SHARED", "")])
        if os.environ.get("BEE_FAULT_DIE_WARM") == "1":
            os._exit(71)  # injected warm-up failure (executor --fault-spawn-fail-rate)
        _cpu_stamp("hello")
        reseed_entropy_state()
        t0 = time.perf_counter()
        warm = os.environ.get("BEE_WARM_GPU") == "1" or bool(os.environ.get("BEE_BROKER_SOCK"))
        gpu_error = warm_gpu() if warm else None
        _cpu_stamp("warm")
        # BEE_PREFAULT=1: exercise the request path's Python machinery while
        # pooled.  Off by default since the request-independent setup moved
        # into the pooled phase: on MI355X it then cost 0.3-0.7 ms of CPU per
        # Execute and bought no latency (profiles/archive/r2_prefault_thp_ab.log)
        if os.environ.get("BEE_PREFAULT", "0") == "1":
            _prefault()
        _prefault_scientific()
        _cpu_stamp("prefault")
        # what the run needs that does not depend on the request, done while
        # pooled: stdout / stderr onto the run's files (opened at boot) and
        # the /workspace view -- the request path then starts the script
        meta = os.environ.get("BEE_META_DIR", "")
        if meta and "stdout" in _OUT_FDS and "stderr" in _OUT_FDS:
            _redirect_stdio(os.path.join(meta, "stdout"), os.path.join(meta, "stderr"))
        _cpu_stamp("redirect")
        rp = os.environ.get("BEE_RUNTIME_PACKAGES", "")
        ws_view, rp_view = _logical_view(cwd, rp)
        _cpu_stamp("view")
        _prepare_paths(rp_view)
        _cpu_stamp("paths")
        chan.send(('{"op":"ready","warm_ms":%.3f,"gpu_error":%s}\n'
                   % ((time.perf_counter() - t0) * 1e3, _json_str(gpu_error or ""))).encode())
        _cpu_stamp("ready")
        _cow_mark()
        job = chan.recv_json()
        if job is None or job.get("op") != "run":
            os._exit(0)
        _STAMPS["recv"] = time.monotonic() * 1e3
        _cow_begin(bool(job.get("cow_trusted")))
        ru = resource.getrusage(resource.RUSAGE_SELF)  # CPU spent while pooled (warm-up, prefault)
        _STAMPS["cpu_pool_ms"] = (ru.ru_utime + ru.ru_stime) * 1e3
        _STAMPS["minflt_pool"] = ru.ru_minflt
        job_env = job.get("env") or {}
        for k, v in job_env.items():
            os.environ[k] = str(v)
        if job.get("numpy_offload") or os.environ.get("BEE_NUMPY_OFFLOAD") == "1":
            _NUMPY_OFFLOAD.append(True)
        _apply_job_quota(int(job.get("hbm_quota") or 0))
        if _REDIRECTED != [job["stdout"], job["stderr"]]:
            _redirect_stdio(job["stdout"], job["stderr"])
        _STAMPS["redir"] = time.monotonic() * 1e3
    except BaseException:
        try:
            traceback.print_exc()
        finally:
            os._exit(70)
    script = job["script"]
    if "TMPDIR" in job_env or "BEE_RUNTIME_PACKAGES" in job_env:  # the request moved what the view maps
        rp = os.environ.get("BEE_RUNTIME_PACKAGES", "")
        ws_view, rp_view = _logical_view(cwd, rp)
    _STAMPS["view"] = time.monotonic() * 1e3
    if ws_view != cwd:
        script = _to_logical(script, cwd, ws_view)
        if rp and rp_view:
            script = _to_logical(script, rp, rp_view)
    code = run_script(script, job.get("argv") or [], ws_view, rp_view, job.get("code"))
    _finish(code, os.path.join(os.path.dirname(job["stdout"]), "timing.json"), chan)
