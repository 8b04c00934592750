"""Device time of each kernel of the headline payload
(examples/benchmark_numpy_gpu.py), in isolation on one MI355X, with the
HBM bytes each must move and the GB/s that implies:

    python tools/payload_kernels.py [--reps 50]

Native driver (this process owns the HIP context); HIP-event timing,
median and min over --reps launches after warm-up."""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bee_code_interpreter_fs_amd import ops as bk  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    bk.synchronize()
    ts = []
    for _ in range(reps):
        with bk.Timer() as t:
            fn()
        ts.append(t.ms * 1e3)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    bk.init(0)
    n = 4096
    a = bk.random.uniform(-1, 1, (n, n), dtype="bfloat16")
    b = bk.random.uniform(-1, 1, (n, n), dtype="bfloat16")
    c = bk.matmul(a, b.T)
    rows = bk.sum(c, axis=1)
    s = bk.sum(b, axis=0).astype("bfloat16").reshape(1, n)
    ref = bk.gemm_bf16_tn(a, s, out_dtype="float32").reshape(n)
    mb = 1 << 20
    big = 10 ** 8
    bk.set_lazy_random(False)
    x = bk.random.rand(big)  # the materialised payload's 800 MB array
    bk.set_lazy_random(True)

    def rand_materialised():
        prev = bk.set_lazy_random(False)
        try:
            return bk.random.rand(big)._materialize()
        finally:
            bk.set_lazy_random(prev)

    cases = [
        ("philox_uniform f64 1e8 (materialised)", rand_materialised, 8 * big, None),
        ("square-sum f64 1e8 (materialised array)", lambda: float(bk.sum(bk.square(x))), 8 * big, None),
        ("philox_uniform_bf16 4096^2", lambda: bk.random.uniform(-1, 1, (n, n), dtype="bfloat16"), 2 * n * n, None),
        ("gemm_bf16_tn 4096^3 (bf16 out)", lambda: bk.matmul(a, b.T), 3 * 2 * n * n, 2 * n ** 3),
        ("rand_reduce f64 1e8 square-sum", lambda: float(bk.sum(bk.square(bk.random.rand(10 ** 8)))), 0, None),
        ("rowsum bf16 4096^2 -> f32", lambda: bk.sum(c, axis=1), 2 * n * n, None),
        ("reduce f32 4096 (checksum)", lambda: float(bk.sum(rows)), 4 * n, None),
        ("colsum bf16 4096^2 -> f32", lambda: bk.sum(b, axis=0), 2 * n * n, None),
        ("cast f32->bf16 4096", lambda: rows.astype("bfloat16"), 6 * n, None),
        ("gemv bf16 4096x4096 . 4096", lambda: bk.gemm_bf16_tn(a, s, out_dtype="float32"), 2 * n * n, 2 * n * n),
        ("max_abs_diff f32 4096", lambda: float(bk.max_abs_diff(rows, ref)), 8 * n, None),
    ]
    total = 0.0
    for name, fn, nbytes, flops in cases:
        med, mn = timed(fn, args.reps)
        total += mn
        rec = {"kernel": name, "us_median": round(med, 2), "us_min": round(mn, 2)}
        if nbytes:
            rec["GBps_at_min"] = round(nbytes / (mn * 1e-6) / 1e9, 1)
            rec["MiB"] = round(nbytes / mb, 2)
        if flops:
            rec["TFLOPs_at_min"] = round(flops / (mn * 1e-6) / 1e12, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"sum_of_mins_us": round(total, 1)}), flush=True)


if __name__ == "__main__":
    main()
