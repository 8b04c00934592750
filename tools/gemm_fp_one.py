"""Run one f64 / f32 GEMM implementation back to back -- beekern's
(csrc/kernels/gemm_fp.hip) or torch.matmul's (rocBLAS / hipBLASLt) -- for
rocprofv3 counter passes (tools/gemm_fp_pmc.sh):

    python tools/gemm_fp_one.py --impl bk|x6|torch --dtype float32 --size 4096 --reps 10

(x6: the f32 product through the six-piece bf16 split, bk_gemm_f32x6)
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_fp_bench import gemm, gemm_x6  # noqa: E402
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--impl", choices=["bk", "x6", "torch"], default="bk")
    p.add_argument("--dtype", default="float32")
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--reps", type=int, default=10)
    a = p.parse_args()
    dt = getattr(torch, a.dtype)
    n = a.size
    x = torch.empty(n, n, device="cuda", dtype=dt).uniform_(-1, 1)
    y = torch.empty(n, n, device="cuda", dtype=dt).uniform_(-1, 1)
    c = torch.empty(n, n, device="cuda", dtype=dt)
    lib = _native.lib()
    ws = torch.empty(lib.bk_gemm_f32x6_workspace_bytes(n, n, n), device="cuda", dtype=torch.uint8)
    for _ in range(a.reps):
        if a.impl == "bk":
            gemm(lib, x, y, c)
        elif a.impl == "x6":
            gemm_x6(lib, x, y, c, ws)
        else:
            torch.matmul(x, y, out=c)
    torch.cuda.synchronize()
    print("done", a.impl, a.dtype, n, a.reps)


if __name__ == "__main__":
    main()
