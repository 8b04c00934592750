"""TFLOP/s of the shipped GEMM dispatch on aligned vs unaligned shapes
(the edge kernels' target: >= 80% of the aligned path), plus hipBLASLt
(torch.matmul) on the same shapes for reference.  One process, events timing."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402

lib = _native.lib()
shapes = [(1024, 1024, 1024), (1000, 1000, 1000), (4096, 4096, 4096), (4095, 4097, 4096), (4000, 4000, 4000),
          (8192, 8192, 8192), (8191, 8193, 8192)]
out = []
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    bt = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    pick = lib.bk_gemm_bf16_pick(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 2)

    def run(variant=0):
        return lib.bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, 2,
                                           variant, s)

    def timeit(fn, iters=50):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    ms = timeit(run)
    ref_ms = timeit(lambda: torch.matmul(a, bt.T, out=c))
    # the 128^2 edge kernel on the same shape, when the 256^2 edge mode was picked
    e6 = timeit(lambda: run(6)) if pick == 7 else None
    fl = 2.0 * M * N * K
    ok = (c.float() - (a.float() @ bt.float().T)).abs().max().item()
    run()
    torch.cuda.synchronize()
    err = (c.float() - (a.float() @ bt.float().T)).abs().max().item() / max(1.0, (a.float() @ bt.float().T).abs().max().item())
    out.append({"shape": [M, N, K], "kernel": pick, "us": round(ms * 1e3, 1), "tflops": round(fl / ms / 1e9, 1),
                "hipblaslt_tflops": round(fl / ref_ms / 1e9, 1), "rel_err": round(err, 5),
                "edge128_tflops": round(fl / e6 / 1e9, 1) if e6 else None})
    print(json.dumps(out[-1]), flush=True)
