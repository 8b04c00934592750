"""bf16 GEMM (bk_gemm_bf16_tn, f32 out) at M = N = 4096 against K: the split
f32 product (bk_gemm_f32x6) runs it at K' = 6 Kp, whose operands (400 MB at
K = 4096) outgrow the 256 MB last-level cache.  Also: the same K' in chunks
accumulated through beta = 1, and torch.matmul (hipBLASLt) at each K.

    python tools/probe/gemm_longk_probe.py
"""

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402


def t(fn, reps=5, rounds=5):
    out = []
    fn()
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / reps * 1e3)
    return statistics.median(out)


def main():
    torch.cuda.init()
    lib = _native.lib()
    st = torch.cuda.current_stream().cuda_stream
    M = N = 4096
    for K in [int(k) for k in os.environ.get("PROBE_KS", "4096 8192 16384 24576").split()]:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = torch.empty(M, N, device="cuda", dtype=torch.float32)

        def bk(kk=K, chunks=1):
            step = kk // chunks
            for i in range(chunks):
                rc = lib.bk_gemm_bf16_tn(a.data_ptr() + 2 * i * step, b.data_ptr() + 2 * i * step, c.data_ptr(), M, N,
                                         step, K, K, N, 1.0, 0.0 if i == 0 else 1.0, 0, st)
                assert rc == 0, rc

        r = {"M": M, "N": N, "K": K, "bk_us": round(t(bk), 1),
             "torch_bf16_us": round(t(lambda: torch.matmul(a, b.T)), 1)}
        r["bk_pflops"] = round(2 * M * N * K / r["bk_us"] / 1e9, 3)
        for v in (4, 5):  # the 256^2 kernel with 8 waves / 4 waves, forced

            def var(v=v):
                rc = lib.bk_gemm_bf16_tn_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0,
                                                 0, v, st)
                assert rc == 0, rc

            r[f"bk_variant{v}_us"] = round(t(var), 1)
        for ch in (2, 3, 6) if os.environ.get("PROBE_CHUNKS", "1") == "1" else ():
            if K % (ch * 64) == 0 and K // ch >= 4096:
                r[f"bk_chunks{ch}_us"] = round(t(lambda ch=ch: bk(K, ch)), 1)
        print(json.dumps(r), flush=True)
        del a, b, c
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
