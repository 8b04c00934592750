"""The headline payload (examples/benchmark_numpy_gpu.py) run in-process on
cuda:0 through beekern's native driver -- the same kernels a served sandbox
reaches through the executor's broker -- so rocprofv3 can trace them:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_payload -o run -- python3 tools/payload_direct.py --iters 20

Prints the payload's own timing per iteration (after one warm-up) and checks
the result like bench.py does.  BEE_LAZY_RANDOM=0 materialises the draw."""

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from bee_code_interpreter_fs_amd import ops as bk

    bk.init(0)
    times, results = [], []
    for it in range(args.iters + 1):
        t0 = time.perf_counter()
        x = bk.random.rand(10**8)
        result = bk.sum(bk.square(x))
        a = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
        b = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
        c = bk.matmul(a, b.T)
        checksum = bk.sum(c)
        r, _ = float(result), float(checksum)
        dt = (time.perf_counter() - t0) * 1e3
        del x, a, b, c
        if it:
            times.append(dt)
            results.append(r)
    ok = all(abs(r - 10**8 / 3) < 5e4 for r in results)
    print(json.dumps({"payload_ms_median": round(statistics.median(times), 3), "payload_ms_min": round(min(times), 3),
                      "iters": args.iters, "lazy_random": os.environ.get("BEE_LAZY_RANDOM", "1"), "result_ok": ok}))


if __name__ == "__main__":
    main()
