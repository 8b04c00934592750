"""Run one bf16 GEMM kernel variant back to back (for rocprofv3 counters).

    python tools/gemm_one.py --variant 3 --size 4096 --reps 50
    python tools/gemm_one.py --nn --size 4096      # the [K][N]-B kernel (bk_gemm_bf16_nn)
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bee_code_interpreter_fs_amd.ops import _native  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", type=int, default=3)
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--k", type=int, default=0)
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--nn", action="store_true", help="B stored [K][N]: bk_gemm_bf16_nn")
    a = p.parse_args()
    n, k = a.size, a.k or a.size
    lib = _native.lib()
    A = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    B = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(a.reps if not a.nn and a.variant != 0 else 0):
        rc = lib.bk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, k, k, k, n, 1.0, 0.0, 2,
                                         a.variant, s)
        assert rc == 0, rc
    for _ in range(a.reps if a.nn else 0):
        rc = lib.bk_gemm_bf16_nn(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, k, k, n, n, 1.0, 0.0, 2, s)
        assert rc == 0, rc
    if a.variant == 0 and not a.nn:
        for _ in range(a.reps):
            torch.matmul(A, B.T, out=C)
    torch.cuda.synchronize()
    print("ok", a)


if __name__ == "__main__":
    main()
