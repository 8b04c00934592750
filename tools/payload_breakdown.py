"""Per-op wall time of the benchmark-numpy GPU payload inside sandboxes, at
several concurrency levels, through the real service (ServiceHarness).  Shows
where in-sandbox time goes (broker round trips, allocation, GPU work)."""

import asyncio
import json
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CODE = r'''
import time
t = [time.perf_counter()]
import beekern as bk
t.append(time.perf_counter())
x = bk.random.rand(10**8); t.append(time.perf_counter())
r = bk.sum(bk.square(x)); t.append(time.perf_counter())
a = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16"); t.append(time.perf_counter())
b = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16"); t.append(time.perf_counter())
c = bk.matmul(a, b.T); t.append(time.perf_counter())
s = bk.sum(c); t.append(time.perf_counter())
ref = bk.dot(bk.sum(a, axis=0), bk.sum(b, axis=0)); t.append(time.perf_counter())
print("Result:", r, s, ref); t.append(time.perf_counter())
del x, a, b, c; t.append(time.perf_counter())
names = ["import", "rand_f64", "square_sum", "rand_bf16_a", "rand_bf16_b", "matmul", "sum_c", "colsum_dot", "print",
         "free"]
print("BREAKDOWN", {n: round((t[i + 1] - t[i]) * 1e3, 3) for i, n in enumerate(names)})
'''


def main():
    from tests.harness import ServiceHarness, ensure_native_executor

    ensure_native_executor()
    h = ServiceHarness(tempfile.mkdtemp(prefix="bee-bd-"), gpu_ids=[0], workers_per_gpu_target=1,
                       min_workers_per_gpu_target=16, light_workers_per_gpu_target=2, max_inflight_per_gpu=64, default_timeout=120.0)
    h.start()
    try:
        for conc in (1, 4, 8, 16):
            async def many():
                ex = h.ctx.code_executor
                out = []
                for _ in range(4):
                    out += await asyncio.gather(*(ex.execute(source_code=CODE) for _ in range(conc)))
                return out
            rs = h.call(many(), timeout=600)
            per = {}
            for r in rs:
                if r.exit_code != 0:
                    print("ERR", r.stderr[-400:])
                    continue
                d = eval(r.stdout.split("BREAKDOWN", 1)[1].strip())
                for k, v in d.items():
                    per.setdefault(k, []).append(v)
            print(json.dumps({"concurrency": conc, **{k: round(statistics.median(v), 3) for k, v in per.items()}}),
                  flush=True)
    finally:
        h.stop()


if __name__ == "__main__":
    main()
