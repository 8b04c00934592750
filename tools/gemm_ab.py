"""bf16 GEMM kernels A/B on one MI355X, in one process (guide §5.4 rule 24):
correctness vs an fp32 torch reference, a race screen (bitwise-identical
repeats: the kernels are deterministic, so any difference is a race), and
interleaved timing rounds of beekern's 128^2 and 256^2 kernels against
torch/hipBLASLt on the same uniform [-1, 1) operands.

    python tools/gemm_ab.py [--rounds 5] [--reps 20]
"""

import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402

VARIANTS = {2: "bk128", 3: "bk256"}


def gemm(lib, a, bt, c, variant):
    M, K = a.shape
    N = bt.shape[0]
    rc = lib.bk_gemm_bf16_tn_variant(
        a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, 2 if c.dtype == torch.bfloat16 else 0,
        variant, torch.cuda.current_stream().cuda_stream,
    )
    if rc != 0:
        raise RuntimeError(f"variant {variant} rc={rc} for {M}x{N}x{K}")


def check(lib, M, N, K, repeats):
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N * 7 + K)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    ref = a.float() @ bt.float().T
    out = {}
    for v, name in VARIANTS.items():
        if v == 3 and (M % 256 or N % 256):
            continue
        c = torch.empty(M, N, device="cuda", dtype=torch.float32)
        gemm(lib, a, bt, c, v)
        torch.cuda.synchronize()
        err = (c - ref).abs().max().item()
        first = c.clone()
        mism = 0
        for _ in range(repeats):
            c.fill_(float("nan"))
            gemm(lib, a, bt, c, v)
            mism += int(not torch.equal(c, first))
        torch.cuda.synchronize()
        out[name] = {"max_abs_err": err, "racy_repeats": mism}
    return out


def bench(lib, size, rounds, reps, k=None):
    k = k or size
    a = torch.empty(size, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    bt = torch.empty(size, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    c = torch.empty(size, size, device="cuda", dtype=torch.bfloat16)
    fns = {name: (lambda v=v: gemm(lib, a, bt, c, v)) for v, name in VARIANTS.items()}
    fns["hipblaslt"] = lambda: torch.matmul(a, bt.T, out=c)
    times = {k: [] for k in fns}
    for f in fns.values():
        for _ in range(3):
            f()
    for _ in range(rounds):
        for name, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                f()
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / reps)
    flops = 2 * size * size * k
    return {
        name: {"us_median": 1e3 * statistics.median(t), "TFLOPs_median": flops / statistics.median(t) / 1e9,
               "TFLOPs_best": flops / min(t) / 1e9}
        for name, t in times.items()
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--repeats", type=int, default=10)
    p.add_argument("--sizes", type=int, nargs="*", default=[4096, 8192])
    p.add_argument("--small-k", type=int, nargs="*", default=[64, 256, 1024])
    p.add_argument("--no-check", action="store_true")
    args = p.parse_args()
    torch.cuda.init()
    lib = _native.lib()
    checks = [] if args.no_check else [(256, 256, 64), (256, 512, 128), (512, 256, 192), (2048, 2048, 320), (4096, 4096, 4096),
                    (1280, 3840, 1088), (8192, 4096, 1024)]
    for M, N, K in checks:
        r = check(lib, M, N, K, args.repeats)
        print(json.dumps({"check": f"{M}x{N}x{K}", **r}), flush=True)
    for size in args.sizes:
        print(json.dumps({"bench": size, **bench(lib, size, args.rounds, args.reps)}), flush=True)
    for k in args.small_k:  # fixed costs (prologue fill, epilogue) at 4096^2
        print(json.dumps({"bench": f"4096x4096x{k}", **bench(lib, 4096, args.rounds, args.reps, k)}), flush=True)


if __name__ == "__main__":
    main()
