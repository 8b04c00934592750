"""The CPU example payloads (examples/*.py) through the full service stack,
the way the reference's e2e suite drives its examples, plus
the ``code_interpreter`` compatibility entry points.  GPU payloads
(benchmark_numpy_gpu, beekern_kernels, torch_on_gpu, allreduce_gang) are
exercised in tests/test_sandbox_gpu.py on the MI355X box.
"""

import os
import subprocess
import sys

import grpc
import pytest

from bee_code_interpreter_fs_amd.models import proto as pb

from .harness import ServiceHarness, ensure_native_executor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES = os.path.join(ROOT, "examples")


def src(name: str) -> str:
    with open(os.path.join(EXAMPLES, name)) as fh:
        return fh.read()


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    ensure_native_executor()
    h = ServiceHarness(str(tmp_path_factory.mktemp("svc")), default_timeout=60.0)
    h.start()
    channel = grpc.insecure_channel(h.grpc_target)
    yield pb.CodeInterpreterServiceStub(channel)
    channel.close()
    h.stop()


def run(stub, name, **kw):
    return stub.Execute(pb.ExecuteRequest(source_code=src(name), **kw), timeout=120)


def test_hello_world(stub):
    r = run(stub, "hello_world.py")
    assert (r.exit_code, r.stdout) == (0, "hello world\n")


def test_write_then_read_file(stub):
    w = run(stub, "write_file.py")
    assert w.exit_code == 0 and set(w.files) == {"/workspace/greeting.txt"}
    r = run(stub, "read_file.py", files=dict(w.files))
    assert r.exit_code == 0 and r.stdout == "Hello, World!\n" and not r.files


def test_workspace_layout(stub):
    w = run(stub, "write_file.py")
    r = run(stub, "workspace_layout.py", files=dict(w.files))
    assert r.stdout.startswith("cwd: /workspace\n"), r.stdout
    assert "greeting.txt" in r.stdout


def test_shell_quoting_is_literal(stub):
    r = run(stub, "shell_quoting.py")
    assert r.exit_code == 0
    assert r.stdout.splitlines() == [
        "single 'quoted' text",
        'double "quoted" text',
        "literal $HOME and ${PATH}",
        "back\\slash",
    ]


def test_division_error(stub):
    r = run(stub, "division_error.py")
    assert r.exit_code == 1 and "ZeroDivisionError" in r.stderr


def test_scientific_stack(stub):
    r = run(stub, "scientific_stack.py")
    assert r.exit_code == 0 and "P-Value" in r.stdout, r.stderr


def test_benchmark_fib(stub):
    r = run(stub, "benchmark_fib.py")
    assert r.exit_code == 0, r.stderr
    assert "digits: 2090" in r.stdout and "Execution Time" in r.stdout


def test_fib_recursive_hits_timeout(stub):
    r = run(stub, "fib_recursive.py", timeout=1.0)
    assert r.exit_code == -1 and "Execution timed out" in r.stderr
    assert r.stdout == ""  # reference shape: ("", "Execution timed out", -1), server.rs:201-218


def test_outbound_socket_reports_outcome(stub):
    r = run(stub, "outbound_socket.py")
    assert r.exit_code == 0
    assert r.stdout.startswith("no egress") or r.stdout.startswith("b'HTTP")


def test_compat_entry_points_import():
    from code_interpreter.config import Config

    assert Config().grpc_listen_addr
    out = subprocess.run(
        [sys.executable, "-c", "import code_interpreter.health_check as h; print(h.health_check.__name__)"],
        cwd=ROOT, capture_output=True, text=True, timeout=120,
    )
    assert out.returncode == 0 and out.stdout.strip() == "health_check", out.stderr


def test_absolute_workspace_paths(stub):
    code = (
        "import os, subprocess, sys\n"
        "open('/workspace/out.txt', 'w').write('x')\n"
        "os.makedirs('/workspace/d', exist_ok=True)\n"
        "open('/workspace/d/y.txt', 'w').write('y')\n"
        "print(os.getcwd(), sorted(os.listdir('/workspace')))\n"
        "print(subprocess.run(['cat', '/workspace/d/y.txt'], capture_output=True, text=True).stdout)\n"
        "print(__file__)\n"
    )
    r = stub.Execute(pb.ExecuteRequest(source_code=code), timeout=60)
    assert r.exit_code == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("/workspace [") and "'out.txt'" in lines[0]
    assert lines[1] == "y"
    assert lines[-1].endswith(".py")
    assert set(r.files) == {"/workspace/out.txt", "/workspace/d/y.txt"} or set(r.files) == {"/workspace/out.txt"}


def test_source_file_traceback_names_workspace_path(tmp_path_factory):
    """HTTP source_file: the script lives in the workspace, and the user sees
    it under /workspace (tracebacks, __file__), as in a reference pod."""
    import httpx

    ensure_native_executor()
    h = ServiceHarness(str(tmp_path_factory.mktemp("svc2")), default_timeout=60.0)
    h.start()
    try:
        with httpx.Client(base_url=h.http_base, timeout=60) as http:
            up = http.put("/v1/files", files={"file": ("div.py", src("division_error.py").encode())})
            sid = up.json()["hash"]
            body = http.post(
                "/v1/execute", json={"source_file": "/workspace/tools/div.py", "files": {"/workspace/tools/div.py": sid}}
            ).json()
    finally:
        h.stop()
    assert body["exit_code"] == 1
    assert 'File "/workspace/tools/div.py", line 3' in body["stderr"], body["stderr"]


# the reference executor image's Python stack (executor/Dockerfile:43-89,
# requirements.txt): each module gets a tiny real use inside a sandbox; a
# module this machine does not have is skipped, not failed (the deploy image,
# deploy/Dockerfile + deploy/requirements-sandbox.txt, installs them all)
STACK = {
    "sympy": "import sympy\nx = sympy.symbols('x')\nprint(sympy.integrate(x**2, (x, 0, 3)))",
    "tabulate": "from tabulate import tabulate\nprint(tabulate([[1, 2]], headers=['a', 'b'], tablefmt='plain').split()[0])",
    "jinja2": "import jinja2\nprint(jinja2.Template('{{ a }}+{{ b }}').render(a=1, b=2))",
    "xarray": "import xarray as xr, numpy as np\nprint(float(xr.DataArray(np.arange(4.0)).sum()))",
    "cv2": "import cv2, numpy as np\nprint(cv2.cvtColor(np.zeros((2, 2, 3), np.uint8), cv2.COLOR_BGR2GRAY).shape)",
    "pikepdf": "import pikepdf\npdf = pikepdf.new(); pdf.add_blank_page(); print(len(pdf.pages))",
    "fitz": "import fitz\nprint(len(fitz.open()))",
    "PyPDF2": "import PyPDF2\nprint(PyPDF2.__version__.split('.')[0])",
    "moviepy": "import moviepy\nprint('moviepy ok')",
    "pdf2image": "import pdf2image\nprint('pdf2image ok')",
    "openpyxl": "import openpyxl\nwb = openpyxl.Workbook(); print(wb.active.title)",
}
EXPECT = {"sympy": "9", "tabulate": "a", "jinja2": "1+2", "xarray": "6.0", "cv2": "(2, 2)", "pikepdf": "1",
          "fitz": "0", "PyPDF2": "2", "moviepy": "moviepy ok", "pdf2image": "pdf2image ok", "openpyxl": "Sheet"}


@pytest.mark.parametrize("module", sorted(STACK))
def test_reference_image_stack(stub, module):
    pytest.importorskip(module)
    r = stub.Execute(pb.ExecuteRequest(source_code=STACK[module]), timeout=120)
    assert r.exit_code == 0, r.stderr
    assert r.stdout.strip() == EXPECT[module], r.stdout


def test_import_to_distribution_and_preinstalled():
    from bee_code_interpreter_fs_amd.runtime import deps

    assert deps.distribution_for("cv2") == "opencv-python-headless"
    assert deps.distribution_for("fitz") == "pymupdf" and deps.distribution_for("yt_dlp") == "yt-dlp"
    assert deps.distribution_for("somethingelse") == "somethingelse"
    # the image's own stack is never re-installed ad hoc (requirements-skip.txt)
    for name in ("ffmpeg-python", "pymupdf", "opencv-python-headless", "PyPDF2", "sympy"):
        assert name in deps.PREINSTALLED
    assert deps.imported_modules("import cv2, os\nfrom fitz import open as o\nimport yt_dlp.utils") == ["cv2", "os", "fitz", "yt_dlp"]


ENV_VIEWS = r"""
import json, os, subprocess
out = subprocess.run(["env", "-0"], capture_output=True).stdout.decode()
libc = dict(kv.split("=", 1) for kv in out.split("\0") if "=" in kv)
# (the path shim hands its mapping to child processes through libc's environment only)
libc = {k: v for k, v in libc.items() if not k.startswith("BEE_FSMAP_")}
py = dict(os.environ)
print(json.dumps({"only_one_side": sorted(set(libc) ^ set(py)),
                  "differ": sorted(k for k in set(libc) & set(py) if libc[k] != py[k]),
                  "tmpdir": py.get("TMPDIR", ""), "home": py.get("HOME", ""),
                  "workspace": py.get("BEE_WORKSPACE", "")}))
"""


def test_sandbox_environment_is_one_view(stub):
    """The sandbox's environment is assembled partly in the zygote (entries
    shared by every spawn) and partly by the native bootstrap (setenv + the
    os.environ mapping): Python's view and what a child process inherits must
    be the same, with the per-sandbox entries present."""
    import json

    r = stub.Execute(pb.ExecuteRequest(source_code=ENV_VIEWS), timeout=120)
    assert r.exit_code == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["only_one_side"] == [] and d["differ"] == [], d
    assert d["tmpdir"] and d["home"] and d["workspace"], d


def test_beekern_only_script_runs_numpy_free(stub):
    """A script importing only beekern + stdlib is served by a sandbox whose
    zygote never imported numpy (executor kind "nano"): numpy is not in
    sys.modules until beekern needs it, and then it still imports
    (ops/_lazy.py): the zygote ran without `site` start-up hooks (python -S)
    yet site-packages stay importable.  (A script importing dynamically --
    __import__, importlib -- goes to a site-enabled sandbox instead.)"""
    src = (
        "import sys, time\n"
        "import beekern as bk\n"
        "print('numpy' in sys.modules, bk.__name__, sys.flags.no_site, 'certifi' in sys.modules)\n"
        "print(bk.normalize_dtype(float))\n"  # beekern imports numpy on first use (ops/_lazy.py)
        "np = sys.modules['numpy']\n"
        "print(np.float64(2.5) * 2)\n"
    )
    r = stub.Execute(pb.ExecuteRequest(source_code=src), timeout=120)
    assert r.exit_code == 0, r.stderr
    assert r.stdout.split("\n")[:3] == ["False bee_code_interpreter_fs_amd.ops 1 False", "float64", "5.0"], r.stdout
    r = stub.Execute(pb.ExecuteRequest(source_code="import sys\nimport numpy, beekern\nprint('numpy' in sys.modules)\n"),
                     timeout=120)
    assert (r.exit_code, r.stdout) == (0, "True\n"), r.stderr


def test_stdlib_only_script_has_the_site_builtins(stub):
    """nano_cpu sandboxes come from a `python -S` zygote: exit() / quit() and
    the other builtins `site` would add still exist."""
    r = stub.Execute(pb.ExecuteRequest(source_code="import sys\nprint(sys.flags.no_site, callable(help))\nexit(3)\n"),
                     timeout=120)
    assert (r.exit_code, r.stdout) == (3, "1 True\n"), (r.stdout, r.stderr)


def test_repeated_source_runs_precompiled_with_the_same_traceback(stub):
    """The second Execute of the same source gets the front-end's
    precompiled code (scheduler/local_gpu_pool.py precompiled_if_repeated):
    output, exit status and the traceback (file name, line, source line)
    are the ones the sandbox's own compile gives."""
    src = "import os\n\ndef f(x):\n    return 1 / x\n\nprint('before', __name__)\nf(0)\n"
    runs = [stub.Execute(pb.ExecuteRequest(source_code=src), timeout=120) for _ in range(3)]
    for r in runs:
        assert r.exit_code == 1 and r.stdout == "before __main__\n", (r.stdout, r.stderr)
        assert 'line 7, in <module>' in r.stderr and 'line 4, in f' in r.stderr, r.stderr
        assert "return 1 / x" in r.stderr and "ZeroDivisionError" in r.stderr, r.stderr
    # same frames, same file, whichever way the code was compiled
    strip = lambda e: [l for l in e.splitlines() if "File " not in l]  # noqa: E731 - tmp script names differ
    assert strip(runs[0].stderr) == strip(runs[1].stderr) == strip(runs[2].stderr)
