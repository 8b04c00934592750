"""A/B of the 256x256 bf16 GEMM schedule variants (tools/gemm_lab/gemm_lab.hip)
in ONE process, interleaved (guide §5.4 rules 19/24), against hipBLASLt on the
same uniform [-1, 1) operands (rule 25).

Per variant: max |err| vs an fp32 torch reference and a race screen
(bitwise-identical repeats -- the kernels are deterministic, so any
difference is a race) on shapes that hit the 1-, 2- and 3-K-tile edge paths;
diagnostic variants (L2-resident operands) are timed only.

    python -m bee_code_interpreter_fs_amd._build gemm-lab   # on the CPU box
    python tools/gemm_lab.py [--rounds 7] [--reps 20]
"""

import argparse
import ctypes
import json
import os
import statistics

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {0: "round1", 1: "keep_b0", 2: "round1_nostagger", 3: "keep_b0_nostagger", 4: "diag_round1_l2", 5: "diag_keep_b0_l2",
         6: "w4", 7: "w4_pinned", 8: "w4_interleaved", 9: "w4_nocarry", 10: "w4_directstore",
         11: "w4_asm_interleaved", 12: "w4_asm_nocarry", 13: "w4_asm_early", 14: "w4_asm_reads_early",
         15: "w4_asm_reads_early_glds_early", 16: "w4_asm_group2", 17: "w4_asm_group8", 18: "w4_asm_group16",
         19: "w4_asm_3bar", 20: "w4_asm_3bar_group8", 21: "w4_asm_3bar_edge",
         22: "w4_asm_3bar_spread", 23: "w4_asm_3bar_spread_edge",
         24: "w4_asm_directstore", 25: "diag_w4_asm_no_epilogue",
         26: "w4_asm_swapab", 27: "w4_asm_swapab_edge", 28: "diag_w4_asm_swapab_no_epilogue",
         29: "w4_asm_altsimd", 30: "w4_asm_altsimd_swapab", 31: "w4_asm_altsimd_early", 32: "diag_w4_asm_stamps", 33: "diag_w4_asm_stamps_noglds",
         34: "diag_w4_asm_stamps_split", 35: "w4_asm_splitglds", 36: "diag_w4_asm_noglds",
         37: "w4_asm_spaced", 38: "diag_w4_asm_stamps_spaced", 39: "w4_asm_spaced_edge", 40: "diag_w4_asm_stamps_mfma_only",
         41: "w4_asm_spaced_csoff", 42: "diag_w4_asm_stamps_spaced_csoff", 43: "w4_asm_twobar", 44: "w4_asm_twobar_edge",
         45: "w4_asm_twobar_g10", 46: "w4_asm_twobar_g12", 47: "w4_asm_spaced_ntstore", 48: "w4_asm_twobar_ntstore",
         49: "w4_asm_twobar_g10_ntstore", 50: "w4_asm_twobar_ntstore_edge",
         51: "diag_twobar_no_vmwait", 52: "diag_twobar_no_bar2", 53: "diag_twobar_no_bar1", 54: "diag_twobar_no_syncs",
         55: "diag_twobar_no_next_reads", 56: "diag_twobar_no_glds", 57: "w4_asm_twobar_g10_swapab",
         58: "w4_asm_twobar_g10_ntstore_reads12", 59: "shipped_group2", 60: "shipped_group8", 61: "shipped_group16"}
DIAG = {4, 5, 25, 28, 32, 33, 34, 36, 38, 40, 42, 51, 52, 53, 54, 55, 56}
PROD = None


def load():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "gemm_lab", "libgemmlab.so"))
    lib.gemmlab_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 7 + [ctypes.c_void_p]
    lib.gemmlab_run.restype = ctypes.c_int
    return lib


def run(lib, v, a, bt, c):
    M, K = a.shape
    N = bt.shape[0]
    rc = lib.gemmlab_run(v, a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, int(c.dtype == torch.bfloat16),
                         torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"variant {v} rc={rc} {M}x{N}x{K}")


def check(lib, variants, M, N, K, repeats):
    g = torch.Generator(device="cuda").manual_seed(M * 131 + N * 7 + K)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    ref = a.float() @ bt.float().T
    out = {}
    for v in variants:
        c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float32)
        run(lib, v, a, bt, c)
        torch.cuda.synchronize()
        err = (c - ref).abs().max().item()
        first = c.clone()
        mism = 0
        for _ in range(repeats):
            c.fill_(float("nan"))
            run(lib, v, a, bt, c)
            mism += int(not torch.equal(c, first))
        torch.cuda.synchronize()
        out[NAMES[v]] = {"max_abs_err": err, "racy_repeats": mism, "ok": bool(err < 1e-3 * K ** 0.5 and mism == 0)}
    return out


def bench(lib, variants, M, N, K, rounds, reps):
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fns = {NAMES[v]: (lambda v=v: run(lib, v, a, bt, c)) for v in variants}
    fns["hipblaslt"] = lambda: torch.matmul(a, bt.T, out=c)
    if PROD is not None:  # the shipped libbeekern 256x256 kernel (built without the lab's flags)
        fns["libbeekern_256"] = lambda: PROD.bk_gemm_bf16_tn_variant(
            a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, 2, 3, torch.cuda.current_stream().cuda_stream)
    for f in fns.values():
        for _ in range(5):
            f()
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for name, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                f()
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / reps)
    flops = 2.0 * M * N * K
    return {name: {"us_median": round(1e3 * statistics.median(t), 2), "us_min": round(1e3 * min(t), 2),
                   "TFLOPs_median": round(flops / statistics.median(t) / 1e9, 1)} for name, t in times.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--repeats", type=int, default=8)
    p.add_argument("--variants", type=int, nargs="*", default=None)
    p.add_argument("--no-check", action="store_true")
    p.add_argument("--stamps", action="store_true", help="kDiagStamps: cycles per K-tile and in its wait + barrier")
    p.add_argument("--one", type=int, default=None, help="only run this variant (-1 = hipBLASLt) --reps times at --size^3 (rocprofv3 passes)")
    p.add_argument("--size", type=int, default=4096, help="--one: M = N = K")
    args = p.parse_args()
    torch.cuda.init()
    lib = load()
    global PROD
    try:
        import sys as _sys
        _sys.path.insert(0, ROOT)
        from bee_code_interpreter_fs_amd.ops import _native
        PROD = _native.lib()
    except Exception:  # noqa: BLE001
        PROD = None
    if args.stamps:
        # kDiagStamps: per wave (loop cycles, cycles in the K-tile wait + barrier, K-tiles)
        for v, size in [(v, size) for v in (38, 42) for size in (4096, 8192)]:
            a = torch.empty(size, size, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            bt = torch.empty(size, size, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            c = torch.zeros(size, size, device="cuda", dtype=torch.float32)
            for _ in range(5):
                run(lib, v, a, bt, c)
            torch.cuda.synchronize()
            nb = (size // 256) ** 2
            st = c.view(torch.int32).flatten()[: nb * 4 * 4].view(nb * 4, 4).cpu().numpy().astype("int64")
            loop, wait = st[:, 0] & 0xFFFFFFFF, st[:, 1] & 0xFFFFFFFF
            h0, nk, h1 = st[:, 2] & 0xFFFFFF, (st[:, 2] >> 24) & 0xFF, st[:, 3] & 0xFFFFFFFF
            print(json.dumps({"stamps": size, "variant": NAMES[v], "waves": int(len(loop)), "k_tiles": int(nk[0]),
                              "loop_cycles_per_ktile_median": float(statistics.median(loop / nk)),
                              "wait_barrier_cycles_per_ktile_median": float(statistics.median(wait / nk)),
                              "wait_fraction_median": float(statistics.median(wait / loop)),
                              "wait_fraction_p90": float(sorted(wait / loop)[int(0.9 * len(loop))]),
                              "half0_cycles_per_ktile_median": float(statistics.median(h0 / nk)),
                              "half1_cycles_per_ktile_median": float(statistics.median(h1 / nk))}), flush=True)
        return
    if args.one is not None:
        n = args.size
        a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        bt = torch.empty(n, n, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        for _ in range(args.reps):
            run(lib, args.one, a, bt, c) if args.one >= 0 else torch.matmul(a, bt.T, out=c)
        torch.cuda.synchronize()
        return
    variants = args.variants if args.variants is not None else list(range(lib.gemmlab_count()))
    real = [v for v in variants if v not in DIAG]
    if not args.no_check:
        for M, N, K in [(256, 256, 64), (256, 512, 128), (512, 256, 192), (512, 512, 256), (2048, 2048, 320),
                        (4096, 4096, 4096), (1280, 3840, 1088), (8192, 4096, 1024)]:
            print(json.dumps({"check": f"{M}x{N}x{K}", **check(lib, real, M, N, K, args.repeats)}), flush=True)
    for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 4096, 64), (4096, 4096, 1024)]:
        print(json.dumps({"bench": f"{M}x{N}x{K}", **bench(lib, variants, M, N, K, args.rounds, args.reps)}), flush=True)


if __name__ == "__main__":
    main()
