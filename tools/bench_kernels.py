"""Kernel microbench on one MI355X: beekern vs torch (hipBLASLt / torch eager).

Prints one JSON line per kernel with device time (HIP events, median of
repeats) and the achieved HBM GB/s or TFLOP/s.  Random operands throughout
(zero-filled inputs read high on MI355X: cdna_hip_programming §5.4 rule 25).
"""

import json
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bee_code_interpreter_fs_amd import ops as bk  # noqa: E402


def timed(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    bk.synchronize()
    times = []
    for _ in range(reps):
        with bk.Timer() as t:
            fn()
        times.append(t.ms)
    return statistics.median(times), min(times)


def torch_timed(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    return statistics.median(times), min(times)


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    bk.init()
    info = bk.device_info()
    emit(kernel="device", **info)
    n = 10**8
    # draws are lazy (generated on first use, fused into a consuming
    # reduction): materialise explicitly to time the generator + HBM write
    x = bk.random.rand(n)._materialize()
    ms, mn = timed(lambda: bk.random.rand(n)._materialize())
    emit(kernel="philox_uniform_f64", n=n, ms=ms, min_ms=mn, GBps=n * 8 / ms / 1e6)
    tx = torch.empty(n, dtype=torch.float64, device="cuda")
    ms_t, _ = torch_timed(lambda: tx.uniform_())
    emit(kernel="torch.uniform_ f64", n=n, ms=ms_t, GBps=n * 8 / ms_t / 1e6)

    ms, mn = timed(lambda: bk.square(x)._materialize())
    emit(kernel="square_f64", n=n, ms=ms, min_ms=mn, GBps=n * 16 / ms / 1e6)
    ms_t, _ = torch_timed(lambda: torch.square(tx))
    emit(kernel="torch.square f64", n=n, ms=ms_t, GBps=n * 16 / ms_t / 1e6)

    ms, mn = timed(lambda: bk.sum(x))
    emit(kernel="sum_f64 (incl. 8B readback)", n=n, ms=ms, min_ms=mn, GBps=n * 8 / ms / 1e6)
    ms, mn = timed(lambda: bk.sum(bk.square(x)))
    emit(kernel="square_sum_f64 fused", n=n, ms=ms, min_ms=mn, GBps=n * 8 / ms / 1e6)
    ms_t, _ = torch_timed(lambda: torch.sum(torch.square(tx)))
    emit(kernel="torch.sum(square) f64", n=n, ms=ms_t, GBps=n * 8 / ms_t / 1e6)

    # the payload's lowering: sum(square(rand(n))) as ONE fused
    # Philox->square->reduce kernel (no HBM traffic; compute-bound generator)
    ms, mn = timed(lambda: bk.sum(bk.square(bk.random.rand(n))))
    emit(kernel="fused rand->square->sum f64 (no HBM)", n=n, ms=ms, min_ms=mn, Gdraws_per_s=n / ms / 1e6)

    # whole benchmark-numpy payload on device (host wall clock, includes readback)
    for _ in range(3):
        bk.sum(bk.square(bk.random.rand(n)))
    t0 = time.perf_counter()
    for _ in range(10):
        r = bk.sum(bk.square(bk.random.rand(n)))
    emit(kernel="benchmark-numpy payload (host wall)", ms=(time.perf_counter() - t0) * 100, result=float(r))

    for size in (4096, 8192):
        a = bk.random.uniform(-1, 1, (size, size), dtype="bfloat16")
        b = bk.random.uniform(-1, 1, (size, size), dtype="bfloat16")
        bt = b.T  # Bt view: kernel reads the buffer as [N, K]
        flops = 2 * size**3
        c_probe = bk.empty((size, size), "bfloat16")
        from bee_code_interpreter_fs_amd.ops import _native

        emit(kernel="gemm dispatch", size=size, variant=_native.lib().bk_gemm_bf16_pick(
            a.ptr, b.ptr, c_probe.ptr, size, size, size, size, size, size, 2), a_mod=a.ptr % 256, c_mod=c_probe.ptr % 256)
        ms, mn = timed(lambda: bk.gemm_bf16_tn(a, b, "bfloat16"), reps=20)
        emit(kernel=f"gemm_bf16_tn {size}^3", ms=ms, min_ms=mn, TFLOPs=flops / ms / 1e9, TFLOPs_best=flops / mn / 1e9)
        bt_buf = bk.empty((size * size + 8,), "bfloat16")
        from bee_code_interpreter_fs_amd.ops.array import driver

        drv = driver()
        ms_tr, mn_tr = timed(lambda: drv.transpose(b.ptr, bt_buf.ptr, size, size, size, size), reps=20)
        emit(kernel=f"transpose_bf16 {size}^2", ms=ms_tr, min_ms=mn_tr, GBps=4 * size * size / ms_tr / 1e6)
        # same copy through the LDS-tiled fallback (taken for a destination
        # that is not 16-B aligned)
        ms_tr, mn_tr = timed(lambda: drv.transpose(b.ptr, bt_buf.ptr + 2, size, size, size, size), reps=20)
        emit(kernel=f"transpose_bf16 tiled fallback {size}^2", ms=ms_tr, min_ms=mn_tr, GBps=4 * size * size / ms_tr / 1e6)
        del bt_buf
        ms2, _ = timed(lambda: bk.matmul(a, b), reps=10)
        emit(kernel=f"bk.matmul (transpose+gemm) {size}^3", ms=ms2, TFLOPs=flops / ms2 / 1e9)
        b32 = b.astype("float32")
        ms3, _ = timed(lambda: bk.matmul(a, b32), reps=10)
        emit(kernel=f"bk.matmul f32 b (fused convert+transpose, gemm) {size}^3", ms=ms3, TFLOPs=flops / ms3 / 1e9)
        from bee_code_interpreter_fs_amd.ops._native import DTYPE_CODES

        bt16 = bk.empty((size, size), "bfloat16")
        ms4, _ = timed(lambda: drv.transpose(b32.ptr, bt16.ptr, size, size, size, size, DTYPE_CODES["float32"]), reps=20)
        emit(kernel=f"transpose_to_bf16 from f32 {size}^2", ms=ms4, GBps=6 * size * size / ms4 / 1e6)
        del b32, bt16
        ta = torch.empty(size, size, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
        tb = torch.empty(size, size, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
        ms_t, mn_t = torch_timed(lambda: ta @ tb.T, reps=20)
        emit(kernel=f"torch.matmul (hipBLASLt) {size}^3", ms=ms_t, TFLOPs=flops / ms_t / 1e9, TFLOPs_best=flops / mn_t / 1e9)
        del bt


if __name__ == "__main__":
    main()
