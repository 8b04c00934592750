"""f64 / f32 GEMM (csrc/kernels/gemm_fp.hip) against torch.matmul in the same
dtype (rocBLAS / hipBLASLt), one MI355X, one process, interleaved rounds.

Reports per size and dtype: median / best TFLOP/s of both, the ratio, the
max relative error of both against an fp64 product (f32 case), and a race
screen (bitwise-identical repeats: the kernel is deterministic).

    python tools/gemm_fp_bench.py [--sizes 2048 4096 8192] [--rounds 5] [--reps 10]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402

CODES = {torch.float64: 1, torch.float32: 0}


def gemm(lib, a, b, c, ta=False, tb=False):
    # a / b are the stored buffers: [K][M] when ta, [N][K] when tb
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    rc = lib.bk_gemm_fp(CODES[a.dtype], int(ta), int(tb), a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K,
                        a.shape[1], b.shape[1], c.shape[1], torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"bk_gemm_fp rc={rc}")


def gemm_x6(lib, a, b, c, ws, ta=False, tb=False):
    """f32 on the bf16 MFMA via the six-piece split (bk_gemm_f32x6)."""
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    rc = lib.bk_gemm_f32x6(int(ta), int(tb), a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, a.shape[1],
                           b.shape[1], c.shape[1], ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"bk_gemm_f32x6 rc={rc}")


def timeit(fn, rounds, reps):
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return out


def bench(lib, dtype, M, N, K, rounds, reps, ta=False, tb=False, x6=False):
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K)
    a = torch.empty((K, M) if ta else (M, K), device="cuda", dtype=dtype).uniform_(-1, 1, generator=g)
    b = torch.empty((N, K) if tb else (K, N), device="cuda", dtype=dtype).uniform_(-1, 1, generator=g)
    aa = a.T if ta else a
    bb = b.T if tb else b
    c = torch.empty(M, N, device="cuda", dtype=dtype)
    ct = torch.empty(M, N, device="cuda", dtype=dtype)
    gemm(lib, a, b, c, ta, tb)
    torch.matmul(aa, bb, out=ct)
    torch.cuda.synchronize()
    ref = aa.double() @ bb.double()
    scale = aa.double().abs() @ bb.double().abs()
    err_bk = ((c.double() - ref).abs() / scale).max().item()
    err_t = ((ct.double() - ref).abs() / scale).max().item()
    first = c.clone()
    racy = 0
    for _ in range(3):
        c.fill_(float("nan"))
        gemm(lib, a, b, c, ta, tb)
        racy += int(not torch.equal(c, first))
    fns = {"beekern": lambda: gemm(lib, a, b, c, ta, tb), "torch": lambda: torch.matmul(aa, bb, out=ct)}
    extra = {}
    if x6 and dtype == torch.float32:
        ws = torch.empty(lib.bk_gemm_f32x6_workspace_bytes(M, N, K), device="cuda", dtype=torch.uint8)
        cx = torch.empty(M, N, device="cuda", dtype=dtype)
        gemm_x6(lib, a, b, cx, ws, ta, tb)
        torch.cuda.synchronize()
        extra["max_rel_err_x6"] = ((cx.double() - ref).abs() / scale).max().item()
        extra["max_abs_rel_to_native_x6"] = ((cx.double() - c.double()).abs() / scale).max().item()
        fns["x6"] = lambda: gemm_x6(lib, a, b, cx, ws, ta, tb)
    for f in fns.values():
        f()
    times = {k: [] for k in fns}
    for _ in range(rounds):  # interleaved: the same clocks for both
        for name, f in fns.items():
            times[name] += timeit(f, 1, reps)
    flops = 2.0 * M * N * K
    r = {"dtype": str(dtype).replace("torch.", ""), "shape": f"{M}x{N}x{K}", "ta": ta, "tb": tb,
         "max_rel_err_beekern": err_bk, "max_rel_err_torch": err_t, "racy_repeats": racy, **extra}
    for name, t in times.items():
        r[f"{name}_us_median"] = round(1e3 * statistics.median(t), 1)
        r[f"{name}_tflops_median"] = round(flops / statistics.median(t) / 1e9, 1)
        r[f"{name}_tflops_best"] = round(flops / min(t) / 1e9, 1)
    r["ratio_median"] = round(statistics.median(times["torch"]) / statistics.median(times["beekern"]), 3)
    if "x6" in times:
        r["ratio_median_x6"] = round(statistics.median(times["torch"]) / statistics.median(times["x6"]), 3)
    return r


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", type=int, nargs="*", default=[2048, 4096, 8192])
    p.add_argument("--dtypes", nargs="*", default=["float64", "float32"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--transposes", action="store_true", help="also A^T and B^T views at the first size")
    p.add_argument("--x6", action="store_true", help="f32: also the six-piece bf16 split (bk_gemm_f32x6)")
    args = p.parse_args()
    torch.cuda.init()
    lib = _native.lib()
    for dt in args.dtypes:
        dtype = getattr(torch, dt)
        for n in args.sizes:
            print(json.dumps(bench(lib, dtype, n, n, n, args.rounds, args.reps, x6=args.x6)), flush=True)
        if args.transposes:
            n = args.sizes[0]
            for ta, tb in ((True, False), (False, True)):
                print(json.dumps(bench(lib, dtype, n, n, n, args.rounds, args.reps, ta, tb, x6=args.x6)), flush=True)
        print(json.dumps(bench(lib, dtype, 4000, 3000, 1000, args.rounds, args.reps, x6=args.x6)), flush=True)


if __name__ == "__main__":
    main()
