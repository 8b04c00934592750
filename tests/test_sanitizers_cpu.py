"""The executor daemon under host sanitizers (SURVEY.md §5.2 plan): the
ASan+UBSan and TSan builds of bee-executor serve a mixed workload —
concurrent executions, staged files and collection, a timeout kill, a
2-rank gang, reservation, status/metrics — and their reports must stay
empty.  The daemon is host code only, so these are plain g++ sanitizers
(GPU sanitizers are not available on the MI355X pool).
"""

import asyncio
import glob
import os

import pytest

from bee_code_interpreter_fs_amd import _build
from bee_code_interpreter_fs_amd.scheduler.executor_process import ExecutorProcess

from .harness import ensure_native_executor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GANG = """
import os
print("rank", os.environ["RANK"], "of", os.environ["WORLD_SIZE"])
"""


def _binary(san: str) -> str:
    path = os.path.join(ROOT, "build", "sanitize", f"bee-executor-{san}")
    _build.build([f"bee-executor-{san}"], verbose=False)
    return path


async def _workload(ex: ExecutorProcess, tmp_path) -> None:
    await ex.wait_ready(1, 180)
    src = tmp_path / "in.txt"
    src.write_text("payload")
    jobs = [
        ex.post("/v1/execute", {"source_code": f"print({i} * 3)", "timeout": 60}, timeout=120) for i in range(6)
    ]
    jobs.append(
        ex.post(
            "/v1/execute",
            {
                "source_code": "print(open('in.txt').read()); open('out.txt', 'w').write('x')",
                "files": {"/workspace/in.txt": str(src)},
                "collect_dir": str(tmp_path),
                "timeout": 60,
            },
            timeout=120,
        )
    )
    jobs.append(ex.post("/v1/execute", {"source_code": "import time; time.sleep(30)", "timeout": 1}, timeout=120))
    rs = await asyncio.gather(*jobs)
    assert all(r.status_code == 200 for r in rs), [r.text for r in rs]
    bodies = [r.json() for r in rs]
    assert [b["stdout"] for b in bodies[:6]] == [f"{i * 3}\n" for i in range(6)]
    assert bodies[6]["stdout"] == "payload\n" and set(bodies[6]["files"]) == {"/workspace/out.txt"}
    assert bodies[7]["exit_code"] == -1
    g = await ex.post("/v1/execute", {"source_code": GANG, "nprocs": 2, "gpus": "", "timeout": 60}, timeout=120)
    assert g.json()["exit_code"] == 0, g.text
    r = await ex.post("/v1/reserve", {"ttl": 5, "wait": 5})
    assert r.status_code == 200
    await ex.post("/v1/release", {})
    assert (await ex.get_json("/v1/status"))["executions"] >= 9
    m = await ex.client.request("GET", "/metrics", None, 10)
    assert m.status_code == 200


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_executor_under_sanitizer(tmp_path, san):
    ensure_native_executor()
    binary = _binary(san)
    logdir = tmp_path / "san"
    logdir.mkdir()
    env = {
        "ASAN_OPTIONS": f"detect_leaks=0:halt_on_error=0:log_path={logdir}/asan",
        "UBSAN_OPTIONS": f"print_stacktrace=1:halt_on_error=0:log_path={logdir}/ubsan",
        "TSAN_OPTIONS": f"halt_on_error=0:second_deadlock_stack=1:log_path={logdir}/tsan",
    }

    async def go():
        ex = ExecutorProcess(f"san-{san}", str(tmp_path / "sb"), gpus="", target=2, binary=binary, extra_env=env)
        await ex.start(timeout=120)
        try:
            await _workload(ex, tmp_path)
        finally:
            await ex.close()

    asyncio.run(go())
    reports = sorted(glob.glob(str(logdir / "*")))
    text = "".join(open(p, errors="replace").read() for p in reports)
    assert not reports, f"{san} reported problems:\n{text[:6000]}"
