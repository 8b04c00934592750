"""Where does a sandbox's script time go?  Runs the bench payload (with
top/bottom wall-clock markers) through the service at concurrency 8 and
compares: payload's own Execution Time, marker-to-marker module time, and the
worker's w_script / run phases."""

import asyncio
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests.harness import ServiceHarness, ensure_native_executor

    src = open(os.path.join(ROOT, "examples", "benchmark_numpy_gpu.py")).read()
    code = "import time as _t\n_T0 = _t.perf_counter()\n" + src + \
        "\nprint('MODULE_MS', (_t.perf_counter() - _T0) * 1e3)\n"
    ensure_native_executor()
    h = ServiceHarness(tempfile.mkdtemp(prefix="bee-wt-"), gpu_ids=[0], workers_per_gpu_target=1,
                       min_workers_per_gpu_target=16, light_workers_per_gpu_target=4, max_inflight_per_gpu=64,
                       default_timeout=120.0)
    h.start()
    try:
        for conc in (1, 8):
            async def many():
                ex = h.ctx.code_executor
                out = []
                for _ in range(6):
                    out += await asyncio.gather(*(ex.execute(source_code=code) for _ in range(conc)))
                return out
            rs = h.call(many(), timeout=600)
            mod, exe, ph = [], [], {}
            for r in rs:
                if r.exit_code != 0:
                    print("ERR", r.stderr[-300:])
                    continue
                mod.append(float(r.stdout.split("MODULE_MS")[1].split()[0]))
                exe.append(float(r.stdout.split("Execution Time:")[1].split()[0]) * 1e3)
                for k, v in (r.timings_ms or {}).items():
                    ph.setdefault(k, []).append(v)
            print(json.dumps({"concurrency": conc, "module_ms": round(statistics.median(mod), 3),
                              "exec_ms": round(statistics.median(exe), 3),
                              **{k: round(statistics.median(v), 3) for k, v in sorted(ph.items())}}), flush=True)
    finally:
        h.stop()


if __name__ == "__main__":
    main()
