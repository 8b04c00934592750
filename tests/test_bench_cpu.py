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
