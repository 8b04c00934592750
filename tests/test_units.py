"""Unit tests of the pure-Python layers (no executor, no GPU)."""

import asyncio
import json
import os

import pytest

from bee_code_interpreter_fs_amd.config import Config
from bee_code_interpreter_fs_amd.models import proto as pb
from bee_code_interpreter_fs_amd.services.custom_tool_executor import (
    CustomToolParseError,
    annotation_to_schema,
    build_tool_script,
    parse_docstring,
    parse_tool,
)
from bee_code_interpreter_fs_amd.services.metrics import Metrics
from bee_code_interpreter_fs_amd.services.multipart import MultipartError, boundary_of, parse_multipart
from bee_code_interpreter_fs_amd.services.storage import Storage
from bee_code_interpreter_fs_amd.utils.retry import async_retry, backoff_delays
from bee_code_interpreter_fs_amd.utils.validation import (
    ValidationError,
    check_file_map,
    is_absolute_path,
    is_hash,
    resolve_logical_path,
    split_logical_path,
)

# ---------------------------------------------------------------- config --


def test_config_defaults_match_reference():
    c = Config(_env={})
    assert c.grpc_listen_addr == "0.0.0.0:50051"
    assert c.http_listen_addr == "0.0.0.0:8000"
    assert c.executor_image == "localhost/bee-code-executor:local"
    assert c.executor_container_resources == {} and c.executor_pod_spec_extra == {}
    assert c.file_storage_path == "./.tmp/files"
    assert c.executor_pod_queue_target_length == 5
    assert c.executor_pod_name_prefix == "code-executor-"
    assert c.grpc_tls_cert is None
    fmt = c.logging_config["formatters"]["standard"]["format"]
    assert fmt == "[%(levelname)s] [%(request_id)s] %(name)s: %(message)s"


def test_config_env_parsing():
    env = {
        "APP_GRPC_LISTEN_ADDR": "127.0.0.1:1",
        "app_executor_pod_queue_target_length": "9",  # case-insensitive
        "APP_EXECUTOR_CONTAINER_RESOURCES": '{"limits": {"amd.com/gpu": 1}}',
        "APP_GRPC_TLS_CERT": "-----BEGIN CERT-----",
        "APP_HTTP_LISTEN_ADDR": "",  # empty is ignored
        "APP_GPU_IDS": "[0, 3]",
        "APP_BROKER_ENABLED": "false",
        "APP_DEFAULT_TIMEOUT": "12.5",
        "OTHER": "x",
    }
    c = Config(_env=env)
    assert c.grpc_listen_addr == "127.0.0.1:1"
    assert c.executor_pod_queue_target_length == 9
    assert c.executor_container_resources == {"limits": {"amd.com/gpu": 1}}
    assert c.grpc_tls_cert == b"-----BEGIN CERT-----"
    assert c.http_listen_addr == "0.0.0.0:8000"
    assert c.gpu_ids == [0, 3]
    assert c.broker_enabled is False
    assert c.default_timeout == 12.5


def test_config_rejects_bad_values():
    with pytest.raises(ValueError):
        Config(_env={"APP_EXECUTOR_POD_QUEUE_TARGET_LENGTH": "many"})
    with pytest.raises(ValueError):
        Config(_env={"APP_EXECUTOR_POD_SPEC_EXTRA": "[1, 2]"})
    with pytest.raises(TypeError):
        Config(_env={}, not_a_field=1)


# ------------------------------------------------------------ validation --


def test_hash_and_path_patterns():
    assert is_hash("abc_DEF-123") and not is_hash("") and not is_hash("a/b") and not is_hash("x" * 256)
    assert is_absolute_path("/workspace/a") and not is_absolute_path("//x") and not is_absolute_path("rel")


@pytest.mark.parametrize(
    "path,root,rel",
    [
        ("/workspace/a.txt", "/workspace", "a.txt"),
        ("/workspace/d/e/f.csv", "/workspace", "d/e/f.csv"),
        ("/runtime-packages/pkg/__init__.py", "/runtime-packages", "pkg/__init__.py"),
        ("/data/x.bin", "/workspace", "data/x.bin"),
    ],
)
def test_split_logical_path(path, root, rel):
    assert split_logical_path(path) == (root, rel)


@pytest.mark.parametrize("bad", ["/workspace/../etc/passwd", "/workspace/./a", "/workspace//a", "/workspace", "relative"])
def test_traversal_rejected(bad):
    with pytest.raises(ValidationError):
        split_logical_path(bad)


def test_resolve_logical_path(tmp_path):
    ws, rp = str(tmp_path / "ws"), str(tmp_path / "rp")
    assert resolve_logical_path("/workspace/a/b", ws, rp) == os.path.join(ws, "a/b")
    assert resolve_logical_path("/runtime-packages/m.py", ws, rp) == os.path.join(rp, "m.py")


def test_check_file_map_collects_errors():
    with pytest.raises(ValidationError) as e:
        check_file_map({"rel": "ok", "/workspace/x": "bad hash!", "/workspace/../y": "ok"})
    assert len(e.value.errors) == 3


# --------------------------------------------------------------- storage --


def test_storage_roundtrip(tmp_path):
    st = Storage(str(tmp_path / "s"))

    async def go():
        h = await st.write(b"hello")
        assert len(h) == 64 and await st.exists(h)
        assert await st.read(h) == b"hello"
        async with st.writer() as w:
            await w.write(b"a" * (3 << 20))
            await w.write(b"b")
        assert await st.size(w.hash) == (3 << 20) + 1
        async with st.reader(w.hash) as r:
            chunks = [c async for c in r.iter_chunks(1 << 20)]
        assert b"".join(chunks)[-1:] == b"b"
        await st.delete(h)
        assert not await st.exists(h)
        with pytest.raises(FileNotFoundError):
            await st.delete(h)
        with pytest.raises(FileNotFoundError):
            await st.read("nope")
        with pytest.raises(FileNotFoundError):
            await st.read("../etc/passwd")

    asyncio.run(go())


def test_storage_adopt_links(tmp_path):
    st = Storage(str(tmp_path / "s"))
    src = tmp_path / "out.txt"
    src.write_text("result")
    oid = st.adopt_file(str(src))
    assert open(st.path_of(oid)).read() == "result"


def test_storage_failed_write_leaves_nothing(tmp_path):
    st = Storage(str(tmp_path / "s"))

    async def go():
        with pytest.raises(RuntimeError):
            async with st.writer() as w:
                await w.write(b"partial")
                raise RuntimeError("client went away")

    asyncio.run(go())
    assert [f for f in os.listdir(st.storage_path) if not f.startswith(".")] == []


def test_storage_ttl_sweep(tmp_path):
    """APP_FILE_STORAGE_TTL_SECONDS retention: objects (written or adopted)
    and abandoned temp files older than the TTL go; younger ones stay."""
    import time

    st = Storage(str(tmp_path / "s"))
    old = asyncio.run(st.write(b"old"))
    src = tmp_path / "made_by_sandbox.txt"
    src.write_text("adopted")
    os.utime(src, (time.time() - 10_000, time.time() - 10_000))  # an old mtime must not count
    adopted = st.adopt_file(str(src))
    stale_tmp = st.temp_path()
    open(stale_tmp, "wb").close()
    now = time.time()
    assert st.sweep(3600, now=now) == 0  # everything was stored just now
    assert st.sweep(3600, now=now + 7200) == 3
    assert not os.path.exists(st.path_of(old)) and not os.path.exists(st.path_of(adopted))
    assert not os.path.exists(stale_tmp)
    fresh = asyncio.run(st.write(b"new"))
    assert st.sweep(3600) == 0 and asyncio.run(st.read(fresh)) == b"new"


def test_storage_ttl_sweeper_task(tmp_path):
    from bee_code_interpreter_fs_amd.application_context import ApplicationContext

    cfg = Config()
    cfg.file_storage_path = str(tmp_path / "files")
    cfg.file_storage_ttl_seconds = 0.5
    ctx = ApplicationContext(cfg, setup_log=False)

    async def go():
        oid = await ctx.file_storage.write(b"x")
        ctx.__dict__["code_executor"] = type("Nop", (), {"start": staticmethod(_anoop), "close": staticmethod(_anoop)})()
        await ctx.start()
        for _ in range(60):
            await asyncio.sleep(0.1)
            if not await ctx.file_storage.exists(oid):
                break
        await ctx.close()
        return await ctx.file_storage.exists(oid)

    assert asyncio.run(go()) is False


async def _anoop():
    return None


# ------------------------------------------------------------ custom tool --


def test_docstring_sections():
    desc, ret, params = parse_docstring(
        """
        Does things.
        Second line: with a colon.

        :param x: first
          continued
        :param y2: second
        :returns: a thing
        :raises ValueError: ignored
        """
    )
    assert desc == "Does things.\nSecond line: with a colon."
    assert params == {"x": "first\n  continued", "y2": "second"}
    assert ret == "a thing"


@pytest.mark.parametrize(
    "ann,schema",
    [
        ("int", {"type": "integer"}),
        ("typing.Optional[int]", {"anyOf": [{"type": "null"}, {"type": "integer"}]}),
        ("list[float]", {"type": "array", "items": {"type": "number"}}),
        ("dict[str, bool]", {"type": "object", "additionalProperties": {"type": "boolean"}}),
        ("Tuple[int, str]", {"type": "array", "minItems": 2, "items": [{"type": "integer"}, {"type": "string"}], "additionalItems": False}),
        ("int | None", {"anyOf": [{"type": "integer"}, {"type": "null"}]}),
        ("Any", {}),
    ],
)
def test_annotation_mapping(ann, schema):
    import ast

    assert annotation_to_schema(ast.parse(ann, mode="eval").body) == schema


def test_parse_errors():
    with pytest.raises(CustomToolParseError) as e:
        parse_tool("def f(:\n  pass")
    assert e.value.errors[0].startswith("Syntax error:")
    with pytest.raises(CustomToolParseError) as e:
        parse_tool("x = 1\ndef f(a: int):\n  pass")
    assert "single function" in e.value.errors[0]
    with pytest.raises(CustomToolParseError) as e:
        parse_tool("def f(a: dict[int, str]):\n  pass")
    assert "Unsupported type" in e.value.errors[0]
    with pytest.raises(CustomToolParseError):
        parse_tool("")


def test_tool_script_runs_locally():
    import subprocess
    import sys

    script = build_tool_script("import math\ndef hyp(a: float, b: float) -> float:\n  print('noise')\n  return math.hypot(a, b)", {"a": 3, "b": 4})
    out = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True)
    assert out.returncode == 0 and json.loads(out.stdout) == 5.0


# ----------------------------------------------------------------- proto --


def test_proto_roundtrip_and_oneof():
    req = pb.ExecuteRequest(source_code="print(1)", executor_id="x", files={"/workspace/a": "h"}, gpus=2)
    assert pb.ExecuteRequest.FromString(req.SerializeToString()) == req
    r = pb.ParseCustomToolResponse(success={"tool_name": "t"})
    assert r.WhichOneof("response") == "success"
    r = pb.ExecuteCustomToolResponse(error={"stderr": "boom"})
    assert r.WhichOneof("response") == "error" and r.error.stderr == "boom"
    names = {m.name for m in pb.code_interpreter.descriptor.services_by_name["CodeInterpreterService"].methods}
    assert names == {"Execute", "ParseCustomTool", "ExecuteCustomTool"}


# ------------------------------------------------------------- multipart --


def test_multipart_streaming_parser():
    boundary = "XyZ123"
    body = (
        f"--{boundary}\r\nContent-Disposition: form-data; name=\"other\"\r\n\r\nignored\r\n"
        f"--{boundary}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"a.bin\"\r\n"
        "Content-Type: application/octet-stream\r\n\r\n"
    ).encode() + b"\r\n--XyZ12 not a boundary\r\n" * 3 + f"\r\n--{boundary}--\r\n".encode()

    async def chunks(n):
        for i in range(0, len(body), n):
            yield body[i : i + n]

    for n in (1, 7, 64, 10_000):
        got = {}

        async def on_part(name, filename, headers):
            got[name] = bytearray()

            async def sink(data):
                got[name] += data

            return sink

        parts = asyncio.run(parse_multipart(chunks(n), boundary, on_part))
        assert parts == 2
        assert bytes(got["other"]) == b"ignored"
        assert bytes(got["file"]) == b"\r\n--XyZ12 not a boundary\r\n" * 3
    assert boundary_of('multipart/form-data; boundary="abc"') == "abc"
    with pytest.raises(MultipartError):
        boundary_of("text/plain")


# ------------------------------------------------------------ retry etc. --


def test_retry_policy():
    assert backoff_delays(3) == [4, 4]
    assert backoff_delays(5, minimum=1, maximum=10) == [1, 2, 4, 8]
    calls = []

    async def nosleep(_):
        return None

    @async_retry((RuntimeError,), attempts=3, sleep=nosleep)
    async def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise RuntimeError("transient")
        return "ok"

    assert asyncio.run(flaky()) == "ok" and len(calls) == 3

    @async_retry((RuntimeError,), attempts=3, sleep=nosleep)
    async def bad():
        raise ValueError("not retried")

    with pytest.raises(ValueError):
        asyncio.run(bad())


def test_metrics_render():
    m = Metrics()
    m.inc("bee_x_total", route="/a")
    m.observe_ms("bee_lat_ms", 3.0, rpc="Execute")
    text = m.render()
    assert 'bee_x_total{route="/a"} 1.0' in text
    assert 'bee_lat_ms_bucket{rpc="Execute",le="5"} 1' in text and "bee_lat_ms_count" in text


def test_sandbox_mode_routing(tmp_path):
    from bee_code_interpreter_fs_amd.scheduler.backend import ExecuteRequest
    from bee_code_interpreter_fs_amd.scheduler.local_gpu_pool import sandbox_mode
    from bee_code_interpreter_fs_amd.services.storage import Storage

    st = Storage(str(tmp_path))
    mode = lambda src: sandbox_mode(ExecuteRequest(source_code=src), st)  # noqa: E731
    assert mode("print(1)") == "nano_cpu"  # stdlib only: numpy-free zygote, lazy broker session
    assert mode("import numpy as np, time, json") == "min_cpu"
    assert mode("import numpy as np, time, json\nimport beekern as bk") == "min"
    assert mode("from bee_code_interpreter_fs_amd import ops") == "nano"
    assert mode("import time\nimport beekern as bk") == "nano"  # numpy-free zygote
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert mode(open(os.path.join(root, "examples", "benchmark_numpy_gpu.py")).read()) == "nano"
    assert mode("import pandas as pd") == "light"
    assert mode("from scipy import stats") == "light"
    assert mode("import torch") == "direct"
    assert mode("import numpy\nimport cupy") == "direct"
    # imports a static scan cannot see go to a site-enabled sandbox (never a
    # `python -S` nano one, where .pth start-up hooks did not run)
    assert mode("import importlib\npd = importlib.import_module('pandas')") == "light"
    assert mode("pd = __import__('pan' + 'das')") == "light"
    assert mode("exec('import pandas as pd')\nprint(pd)") == "light"
    assert mode("import beekern as bk\nmod = __import__('json')") == "light"
    assert mode("import torch\nimport importlib") == "direct"
    # methods named like the builtins are no dynamic import:
    # re.compile / obj.eval stay on the numpy-free sandboxes
    assert mode("import re\nprint(re.compile('a+').match('aa'))") == "nano_cpu"
    assert mode("import numpy as np\nclass M:\n    def eval(self): return 1\nM().eval()") == "min_cpu"
    assert mode("code = compile('1 + 1', 'x', 'eval')") == "light"
    # ... but the builtins reached through the builtins module are
    assert mode("import builtins\nbuiltins.exec('import pandas')") == "light"
    assert mode("import builtins\npd = builtins.__import__('pandas')") == "light"
    assert mode("__builtins__.eval('1')") == "light"
    assert mode("f = __builtins__['__import__']") == "light"
    assert mode("import builtins\nprint(builtins.len([1]))") == "nano_cpu"


def test_philox_reference_known_answers():
    """tests/philox_ref.py (the host reference the GPU RNG is checked
    against bit for bit) reproduces the Random123 philox4x32-10 vectors."""
    import numpy as np

    from .philox_ref import philox4x32_10

    def one(ctr, key):
        return [int(w[0]) for w in philox4x32_10(*[np.array([c], dtype=np.uint64) for c in ctr], *key)]

    assert one((0, 0, 0, 0), (0, 0)) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert one((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert one((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_job_quota_reaches_a_lazy_broker_session(monkeypatch):
    """worker._apply_job_quota with a broker-backed (lazy) beekern session:
    the client learns the run's quota (regression: a name clash with the
    package's `array` function made every GPU-slot run exit 70)."""
    import sys

    from bee_code_interpreter_fs_amd import ops
    from bee_code_interpreter_fs_amd.runtime import worker

    arr = sys.modules["bee_code_interpreter_fs_amd.ops.array"]
    monkeypatch.setenv("BEE_BROKER_SOCK", "/nonexistent/broker.sock")
    monkeypatch.setenv("BEE_HBM_QUOTA_BYTES", "0")  # restored after the test
    monkeypatch.setattr(arr, "_driver", None)
    ops.init(0, lazy=True)
    try:
        worker._apply_job_quota(123 << 20)
        assert ops.driver_name() == "broker"
        assert arr.driver().quota == 123 << 20
        assert os.environ["BEE_HBM_QUOTA_BYTES"] == str(123 << 20)
    finally:
        monkeypatch.setattr(arr, "_driver", None)


def test_request_env_allow_list():
    """Gang / custom env: RCCL and torch knobs pass, anything that could
    steer the sandbox bootstrap (jail, quota, pin, loader) is refused."""
    from bee_code_interpreter_fs_amd.scheduler.backend import ExecuteRequest
    from bee_code_interpreter_fs_amd.utils.validation import ValidationError

    ok = ExecuteRequest(source_code="x", env={"NCCL_MIN_NCHANNELS": "16", "RCCL_MSCCL_ENABLE": "0",
                                              "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1", "OMP_NUM_THREADS": "4"}).validate()
    assert ok.env["NCCL_MIN_NCHANNELS"] == "16"
    for bad in ({"BEE_JAIL": "0"}, {"LD_PRELOAD": "/x.so"}, {"HIP_VISIBLE_DEVICES": "0,1"}, {"PYTHONPATH": "/x"},
                {"BEE_HBM_QUOTA_BYTES": "0"}, {"A=B": "1"}, {"HSA_TOOLS_LIB": "x"}):
        with pytest.raises(ValidationError):
            ExecuteRequest(source_code="x", env=bad).validate()


def _fake_sysfs(root, gpus_numa):
    """KFD topology (one CPU node, then GPU nodes) + PCI numa_node + node cpulists."""
    import os

    base = os.path.join(root, "class", "kfd", "kfd", "topology", "nodes")
    os.makedirs(os.path.join(base, "0"))
    open(os.path.join(base, "0", "properties"), "w").write("cpu_cores_count 64\nsimd_count 0\n")
    for i, numa in enumerate(gpus_numa):
        d = os.path.join(base, str(i + 1))
        os.makedirs(d)
        bus = 0x10 + 0x10 * i
        open(os.path.join(d, "properties"), "w").write(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        pci = os.path.join(root, "bus", "pci", "devices", f"0000:{bus:02x}:00.0")
        os.makedirs(pci)
        open(os.path.join(pci, "numa_node"), "w").write(f"{numa}\n")
    for node, cpus in ((0, "0-3,8-11"), (1, "4-7,12-15")):
        d = os.path.join(root, "devices", "system", "node", f"node{node}")
        os.makedirs(d)
        open(os.path.join(d, "cpulist"), "w").write(cpus + "\n")


def test_numa_topology_and_slot_cpus(tmp_path):
    from bee_code_interpreter_fs_amd.scheduler import topology as t

    assert t.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert t.format_cpulist([11, 10, 8, 3, 2, 1, 0]) == "0-3,8,10-11"
    _fake_sysfs(str(tmp_path), [0, 0, 0, 0, 1, 1, 1, 1])
    assert t.gpu_numa_nodes(str(tmp_path)) == [0, 0, 0, 0, 1, 1, 1, 1]
    assert t.slot_cpus(0, str(tmp_path), allowed=set(range(16)), quota=0) == [0, 1, 2, 3, 8, 9, 10, 11]
    assert t.slot_cpus(6, str(tmp_path), allowed=set(range(16)), quota=0) == [4, 5, 6, 7, 12, 13, 14, 15]
    assert t.slot_cpus(6, str(tmp_path), allowed={0, 1, 5}, quota=0) == [5]  # only CPUs this process may use
    assert t.slot_cpus(None, str(tmp_path)) == []


def test_numa_single_node_means_no_pinning(tmp_path):
    from bee_code_interpreter_fs_amd.scheduler import topology as t

    _fake_sysfs(str(tmp_path), [0, 0])
    assert t.slot_cpus(1, str(tmp_path), allowed=set(range(16)), quota=0) == []


def test_cpu_quota_and_quota_pinning(tmp_path):
    """A 16-CPU cgroup quota on a 256-CPU host: the service is pinned to 2x
    the quota, physical cores first, split between the GPU slots."""
    from bee_code_interpreter_fs_amd.scheduler import topology as t

    cg = tmp_path / "cg"
    (cg / "job" / "leaf").mkdir(parents=True)
    (cg / "cpu.max").write_text("max 100000\n")
    (cg / "job" / "cpu.max").write_text("1600000 100000\n")
    (cg / "job" / "leaf" / "cpu.max").write_text("max 100000\n")
    pc = tmp_path / "proc_cgroup"
    pc.write_text("0::/job/leaf\n")
    assert t.cpu_quota(str(cg), str(pc)) == 16.0
    pc.write_text("12:cpu:/x\n")  # cgroup v1 only, no quota files
    assert t.cpu_quota(str(cg), str(pc)) == 0.0
    # a host of 256 logical CPUs, 128 cores: cpu c and c+128 are siblings, one NUMA node
    sys_ = tmp_path / "sys"
    for c in range(256):
        d = sys_ / "devices" / "system" / "cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        d.joinpath("thread_siblings_list").write_text(f"{c % 128},{c % 128 + 128}\n")
    allowed = set(range(256))
    one = t.slot_cpus(0, str(sys_), allowed=allowed, slots=[0], quota=16.0)
    assert one == list(range(32)), one  # 32 physical cores, no SMT siblings
    two = [t.slot_cpus(g, str(sys_), allowed=allowed, slots=[0, 1], quota=16.0) for g in (0, 1)]
    assert two == [list(range(16)), list(range(16, 32))], two
    assert t.slot_cpus(0, str(sys_), allowed=allowed, slots=[0], quota=16.0, factor=0) == []  # off: NUMA rules only
    assert t.slot_cpus(0, str(sys_), allowed=set(range(24)), slots=[0], quota=16.0) == []  # quota ~ what may run
    assert t.core_order([0, 128, 1, 129], str(sys_)) == [0, 1, 128, 129]
    assert t.gpu_numa_nodes(str(tmp_path / "missing")) == []


def test_beekern_imports_without_numpy_and_fill_patterns_match():
    """ops/_lazy.py: importing beekern does not import numpy (the nano
    zygote's premise), and full()'s struct-built fill patterns equal the
    numpy-built ones (bf16: round to nearest even, NaN -> 0x7FC0)."""
    import math
    import struct
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", "import sys; import bee_code_interpreter_fs_amd.ops as o; "
                          "print('numpy' in sys.modules, o.sum.__module__)"], cwd=root, capture_output=True, text=True)
    assert out.stdout.split() == ["False", "bee_code_interpreter_fs_amd.ops.array"], out.stderr

    import numpy as np

    from bee_code_interpreter_fs_amd.ops import _lazy
    from bee_code_interpreter_fs_amd.ops.array import _f32_bits_to_bf16, _f32_to_bf16_bits

    vals = [0.0, -0.0, 1.0, -1.5, 3.14159, 1e-40, 65504.0, 1.00390625, 1.01171875, 3.4e38, math.inf, -math.inf,
            math.nan, 0.1, -2.71828]
    ref = _f32_to_bf16_bits(np.array(vals, np.float32))
    got = [_f32_bits_to_bf16(struct.unpack("<I", struct.pack("<f", v))[0]) for v in vals]
    assert got == [int(x) for x in ref]
    assert _lazy.scalar(1.5) == 1.5 and isinstance(_lazy.scalar(1.5), np.float64)  # numpy loaded here
    assert _lazy.is_number(np.float32(2)) and _lazy.is_integer(np.int64(3)) and not _lazy.is_integer(2.0)


def test_precompiled_payload_roundtrip():
    """The front-end's precompiled payload (local_gpu_pool.precompiled) loads
    in the worker as the code compile(source, path) gives -- every nested code
    object renamed to the sandbox's script path -- and anything odd falls
    back to the worker's own compile (None)."""
    import types

    from bee_code_interpreter_fs_amd.runtime.worker import load_precompiled
    from bee_code_interpreter_fs_amd.scheduler.local_gpu_pool import precompiled

    src = "def f(x):\n    return [i * x for i in range(3)]\nprint(f(2))\n"
    blob = precompiled(src)
    code, shell = load_precompiled(blob, "/workspace/main.py")
    ref = compile(src, "/workspace/main.py", "exec", dont_inherit=True)
    assert not shell and code.co_code == ref.co_code

    def names(c):
        yield c.co_filename
        for k in c.co_consts:
            if isinstance(k, types.CodeType):
                yield from names(k)

    assert set(names(code)) == {"/workspace/main.py"}
    assert precompiled("print(\n") is None  # the sandbox reports the SyntaxError itself
    # a compile that warns stays in the sandbox (its stderr shows the warning
    # on every run, not the front-end's on the repeated ones)
    assert precompiled("x = 1\nassert (x, 'always true')\n") is None
    assert precompiled("x = 1\nprint(x is 1)\n") is None
    assert load_precompiled(precompiled("echo hi\n"), "/x.py")[1] is True  # xonsh-lowered
    assert load_precompiled("not base64 !", "/x.py") is None
    assert load_precompiled(__import__("base64").b64encode(b"\0\0\0\0P...").decode(), "/x.py") is None


def test_precompile_only_repeated_sources():
    from bee_code_interpreter_fs_amd.scheduler import local_gpu_pool as lgp

    src = "print('precompile-once-%d')\n" % os.getpid()
    assert lgp.precompiled_if_repeated(src) is None  # first sight: the sandbox compiles
    assert lgp.precompiled_if_repeated(src) == lgp.precompiled(src)  # seen before: shipped compiled


def test_wait_warm_accepts_a_disabled_warm_gang_set():
    """A warm gang set the daemon gave up on ("disabled") does not hold the
    service's READY back; one still "warming" does (until the timeout)."""
    from types import SimpleNamespace

    from bee_code_interpreter_fs_amd.scheduler.local_gpu_pool import LocalGpuPoolBackend

    def backend(gang_state):
        st = {"zygotes_alive": 1, "zygotes": 1, "ready_direct": 1, "target": 1, "gang_warm": {"0,1": gang_state}}

        async def get_json(path):
            return st

        b = LocalGpuPoolBackend.__new__(LocalGpuPoolBackend)
        b.slots = [SimpleNamespace(executor=SimpleNamespace(get_json=get_json))]
        return b

    assert asyncio.run(backend("ready").wait_warm(1.0)) is True
    assert asyncio.run(backend("disabled").wait_warm(1.0)) is True
    assert asyncio.run(backend("warming").wait_warm(0.3)) is False


def test_load_table_torn_read_keeps_the_last_load(tmp_path):
    """A reader that only ever sees a write in progress (odd seq) returns
    the last load it read, not "no table" -- which routing would take for
    an idle GPU (scheduler/load_table.py)."""
    import struct

    from bee_code_interpreter_fs_amd.scheduler import load_table as lt

    path = tmp_path / "load"
    vals = [lt.MAGIC, 2, 3, 1, 5 << 20, 8, 40 << 30, 0, 17, 1234, 4, 6 << 20]
    path.write_bytes(struct.pack(lt._FMT, *vals).ljust(4096, b"\0"))
    t = lt.open_table(str(path))
    got = t.read()
    assert got is not None and (got.jobs, got.waiting, got.executions, got.depth) == (3, 1, 17, 4)
    with open(path, "r+b") as f:  # the writer stops between its two seq bumps
        f.seek(8)
        f.write(struct.pack("<Q", 3))
        f.seek(16)
        f.write(struct.pack("<q", 7))  # (a half-written jobs count)
    again = t.read()
    assert again is not None and again.jobs == 3 and again.executions == 17
    with open(path, "r+b") as f:  # a table that is not (or no longer) one
        f.write(struct.pack("<QQ", 0, 4))
    assert t.read() is None
    t.close()
