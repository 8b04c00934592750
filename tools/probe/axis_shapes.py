"""Column / row sums of bf16 matrices of growing height (fixed 4096 columns):
separates a kernel's fixed cost (launch, ticket, fold) from its streaming
rate.  Run under rocprofv3 --kernel-trace --stats."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bee_code_interpreter_fs_amd import ops as bk  # noqa: E402

bk.init(0)
for rows in (256, 1024, 4096, 16384):
    x = bk.random.uniform(-1, 1, (rows, 4096), dtype="bfloat16")
    for _ in range(20):
        bk.sum(x, axis=0)
        bk.sum(x, axis=1)
    bk.synchronize()
    print(rows, "done", flush=True)
