"""Fixed vs per-K-tile cost of the shipped 256x256 4-wave GEMM (variant 5):
time M = N = 4096 at K = 64 ... 4096; the intercept is the prologue +
epilogue every tile pays (what a persistent / overlapped epilogue could
recover), the slope the main loop's cost per K-tile."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402

lib = _native.lib()
M = N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
s = torch.cuda.current_stream().cuda_stream
rows = []
for K in (64, 128, 256, 512, 1024, 2048, 4096):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    bt = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for out, dt in ((2, torch.bfloat16), (0, torch.float32)):
        c = torch.empty(M, N, device="cuda", dtype=dt)
        run = lambda: lib.bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0,
                                                  out, 5, s)
        assert run() == 0
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        ref_ms = None
        if out == 2:
            for _ in range(3):
                torch.matmul(a, bt.T, out=c)
            e0.record()
            for _ in range(50):
                torch.matmul(a, bt.T, out=c)
            e1.record()
            torch.cuda.synchronize()
            ref_ms = e0.elapsed_time(e1) / 50
        rows.append({"M": M, "N": N, "K": K, "out": "bf16" if out == 2 else "f32", "us": round(us, 2),
                     "tflops": round(2.0 * M * N * K / us / 1e6, 1),
                     "hipblaslt_us": round(ref_ms * 1e3, 2) if ref_ms else None})
        print(json.dumps(rows[-1]), flush=True)
