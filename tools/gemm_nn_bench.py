"""C = A . B with B row-major [K][N]: the [K][N] kernel (bk_gemm_bf16_nn)
vs the transpose + TN path it replaces vs the TN kernel on a pre-transposed
B vs hipBLASLt (torch.matmul(a, b)).  TFLOP/s, one process, event timing."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402

lib = _native.lib()
s = torch.cuda.current_stream().cuda_stream


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


# shapes: argv[1] as JSON [[M, N, K], ...], default the three README shapes
SHAPES = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [[4096, 4096, 4096], [8192, 8192, 8192], [4096, 8192, 2048]]
for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    bt = b.T.contiguous()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    scratch = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    nn = lambda: lib.bk_gemm_bf16_nn(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, K, N, N, 1.0, 0.0, 2, s)
    assert nn() == 0
    torch.cuda.synchronize()
    err = (c.float() - (a.float() @ b.float())).abs().max().item() / (a.float() @ b.float()).abs().max().item()
    tn = lambda: lib.bk_gemm_bf16_tn(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, 2, s)

    def tr_tn():
        lib.bk_transpose_bf16(b.data_ptr(), scratch.data_ptr(), K, N, N, K, s)
        lib.bk_gemm_bf16_tn(a.data_ptr(), scratch.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, 2, s)

    row = {"shape": [M, N, K], "nn_tflops": round(fl / timeit(nn) / 1e9, 1),
           "transpose_tn_tflops": round(fl / timeit(tr_tn) / 1e9, 1), "tn_tflops": round(fl / timeit(tn) / 1e9, 1),
           "hipblaslt_nn_tflops": round(fl / timeit(lambda: torch.matmul(a, b, out=c)) / 1e9, 1),
           "nn_rel_err": round(err, 5)}
    print(json.dumps(row), flush=True)
