"""bench.py's contract on CPU: offered load grows with --gpus N in a
single-process run (N load-generator processes of --concurrency clients),
pods are labelled by what really runs, and the JSON carries the per-GPU and
CPU fields.  A virtual-GPU rehearsal (executors pinned to GPU ids that need
not exist) stands in for the driver's 8-GPU node."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_single_process_multi_gpu_run_scales_offered_load():
    p = subprocess.run(
        [sys.executable, "bench.py", "--gpus", "2", "--virtual-gpus", "--workload", "hello", "--steps", "4",
         "--warmup", "1", "--concurrency", "3", "--no-gang-check"],
        cwd=ROOT, capture_output=True, text=True, timeout=600,
    )
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and out["errors"] == 0, out
    assert out["completed"] == 2 * 3 * 4  # 2 load generators x 3 clients x 4 steps
    assert out["config"]["global_batch"] == 6
    assert "2 virtual-GPU (CPU rehearsal) executor pods" in out["config"]["parallelism"]
    assert "2 load-generator processes" in out["config"]["parallelism"]
    assert out["per_gpu_rps"] == round(out["value"] / 2, 3)
    assert out["cpu_cores_busy"]["value"] > 0
    assert {"metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling"} <= set(out)


def test_torchrun_two_ranks_one_json_line():
    """The driver's N>1 launch (``torch.distributed.run --nproc-per-node N
    ... bench.py --gpus N``): rank 0 starts the service, every rank drives
    its own clients, the timed window is the max over ranks, and only rank 0
    prints -- one JSON line with the whole job's aggregate."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
         "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--virtual-gpus", "--workload", "hello",
         "--steps", "4", "--warmup", "1", "--concurrency", "3", "--no-gang-check"],
        cwd=ROOT, env=env, capture_output=True, text=True, timeout=600,
    )
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [line for line in p.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["errors"] == 0 and out["completed"] == 2 * 3 * 4, out
    assert out["steps"] == 4 and out["warmup"] == 1 and out["scaling"] == "weak"
    assert abs(out["value"] - out["completed"] / (out["ms_per_step"] * out["steps"] / 1e3)) < 0.05 * out["value"]


def _bf16(x):
    """Round float32 to bfloat16 (nearest even), back as float32."""
    import numpy as np

    b = np.asarray(x, dtype=np.float32).view(np.uint32)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return b.astype(np.uint32).view(np.float32)


def test_headline_checks_bite():
    """the payload's checks, emulated on the host.

    * Result (sum of 1e8 U^2) is accepted within 6 sigma (sigma = sqrt(n *
      4/45) ~ 2981), not the old +-5e4 (~17 sigma);
    * the GEMM check compares every row sum of C = bf16(A @ B.T) with
      A @ bf16(colsum(B)): a correct 4096^3 bf16 GEMM passes with a wide
      margin, one zeroed 256x256 tile fails."""
    import numpy as np

    sys.path.insert(0, ROOT)
    import bench

    assert 2900 < bench.RESULT_SIGMA < 3050
    assert bench.result_ok(bench.EXPECTED + 5.9 * bench.RESULT_SIGMA)
    assert not bench.result_ok(bench.EXPECTED + 6.1 * bench.RESULT_SIGMA)
    assert not bench.result_ok(bench.EXPECTED - 2e4) and not bench.result_ok(0.0)

    rng = np.random.default_rng(7)
    n = 4096
    a = _bf16(rng.uniform(-1, 1, (n, n)).astype(np.float32))
    b = _bf16(rng.uniform(-1, 1, (n, n)).astype(np.float32))
    c = _bf16(a @ b.T)                                   # f32 accumulate, bf16 out
    s = _bf16(b.sum(axis=0, dtype=np.float64).astype(np.float32))  # colsum(B), f64-accumulated, bf16 row
    ref = a.astype(np.float64) @ s.astype(np.float64)
    err = np.abs(c.sum(axis=1, dtype=np.float64) - ref).max()
    assert bench.gemm_row_ok(err) and err < bench.GEMM_ROW_TOL / 4, err
    bad = c.copy()
    bad[256:512, 1024:1280] = 0.0                        # one corrupt tile
    err_bad = np.abs(bad.sum(axis=1, dtype=np.float64) - ref).max()
    assert not bench.gemm_row_ok(err_bad), err_bad


def test_gang_check_is_bounded_and_stops_at_the_first_failure(monkeypatch):
    """The gang check runs after the timed window on the driver's multi-GPU
    node; a gang that fails (or hangs) must not eat the run: the first
    failing run ends it, and one time budget bounds all of them."""
    import importlib.util
    import time
    import types

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    calls = []

    class Stub:
        def __init__(self, ch):
            pass

        def Execute(self, req, timeout):  # noqa: N802 - the gRPC method name
            calls.append((req.timeout, timeout))
            return types.SimpleNamespace(exit_code=1, stdout="", stderr="rccl init failed", timings_ms={})

    class Chan:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    import grpc

    from bee_code_interpreter_fs_amd.models import proto as pb

    monkeypatch.setattr(grpc, "insecure_channel", lambda target: Chan())
    monkeypatch.setattr(pb, "CodeInterpreterServiceStub", Stub)
    t = time.monotonic()
    out = bench.gang_allreduce_check("127.0.0.1:1", 8, repeats=2, hport=None)
    assert time.monotonic() - t < 5
    assert len(calls) == 1 and not out["ok"], out  # no second try of a failing gang
    assert out["runs"][0]["stderr_tail"].endswith("rccl init failed")
    assert calls[0][0] <= 180 and calls[0][1] <= 240  # script and RPC bounded by the budget

    calls.clear()
    monkeypatch.setenv("BEE_BENCH_GANG_BUDGET_S", "10")
    out = bench.gang_allreduce_check("127.0.0.1:1", 8, repeats=2, hport=None)
    assert calls == [] and "budget" in out.get("skipped", ""), out


def test_cpu_throttle_reads_both_cgroup_versions(tmp_path):
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    v2 = tmp_path / "v2.stat"
    v2.write_text("usage_usec 10\nnr_periods 40\nnr_throttled 3\nthrottled_usec 25000\n")
    v1 = tmp_path / "v1.stat"
    v1.write_text("nr_periods 7\nnr_throttled 1\nthrottled_time 2000000\n")
    a = bench.cpu_throttle(((str(tmp_path / "missing"), 1.0), (str(v2), 1.0)))
    assert a == {"periods": 40, "throttled": 3, "throttled_ms": 25.0}
    b = bench.cpu_throttle(((str(v1), 1e-3),))
    assert b == {"periods": 7, "throttled": 1, "throttled_ms": 2.0}
    assert bench.cpu_throttle(((str(tmp_path / "missing"), 1.0),)) == {}
    d = bench.throttle_delta(a, {"periods": 50, "throttled": 5, "throttled_ms": 40.0})
    assert d == {"periods": 10, "throttled_periods": 2, "throttled_ms": 15.0}
    assert bench.throttle_delta({}, a) is None


# the keys a multi-GPU bench line carries (VERDICT r4 "next" #5): the driver's
# first run on the 8-GPU node must explain itself without another run
N_GPU_KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "p50_latency_ms", "completed", "errors", "per_gpu_rps",
              "cpu_bound_rps", "node_bound", "executors", "slot_balance", "gang_allreduce"}
GANG_KEYS = {"gpus", "budget_GBps", "runs", "ok", "busbw_GBps", "busbw_of_budget", "busbw_by_size", "rccl_env",
             "transport", "budget_s"}


import pytest  # noqa: E402


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_gpu_bench_path_end_to_end_with_the_gang_check(n):
    """The whole N-GPU bench path on N virtual GPU slots: load over every
    slot, then the gang check -- an N-rank all-reduce sandbox through the
    service (gloo on CPU where the node runs RCCL) with its per-size bus
    bandwidth against the budget, the collective environment the ranks saw,
    and its time budget -- and the JSON schema of an N > 1 line."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env["BEE_BENCH_GANG_BUDGET_S"] = "200"
    p = subprocess.run(
        [sys.executable, "bench.py", "--gpus", str(n), "--virtual-gpus", "--workload", "hello", "--steps", "3",
         "--warmup", "1", "--concurrency", "2", "--idle-probe", "0"],
        cwd=ROOT, env=env, capture_output=True, text=True, timeout=900,
    )
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([line for line in p.stdout.splitlines() if line.startswith("{")][-1])
    missing = N_GPU_KEYS - set(out)
    assert not missing, (missing, sorted(out))
    assert out["n_gpus"] == n and out["errors"] == 0 and out["completed"] == n * 2 * 3, out
    assert out["cpu_bound_rps"] == out["node_bound"].get("cpu_bound_rps")
    g = out["gang_allreduce"]
    assert not (GANG_KEYS - set(g)), (GANG_KEYS - set(g), g)
    assert g["ok"] and g["gpus"] == n and g["transport"].startswith("gloo"), g
    assert [s["bytes"] for s in g["busbw_by_size"]] == [1 << 16, 1 << 20, 16 << 20], g["busbw_by_size"]
    assert all(s["busbw_GBps"] > 0 and s["of_budget"] == round(s["busbw_GBps"] / g["budget_GBps"], 3)
               for s in g["busbw_by_size"])
    assert g["rccl_env"]["backend"] == "gloo" and g["rccl_env"]["env"].get("NCCL_IB_DISABLE") == "1", g["rccl_env"]
    assert g["budget_s"] == 200.0
    assert all(r["rank_start"] in ("warm", "cold") for r in g["runs"]), g["runs"]
    assert len(out["slot_balance"]["executions"]) == n
