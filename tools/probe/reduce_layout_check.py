"""Numerics of one reduction layout (BK_REDUCE_LAYOUT) against fp64 numpy on
ragged sizes, every single-operand op and dtype:

    BK_REDUCE_LAYOUT=ldsdma python tools/probe/reduce_layout_check.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bee_code_interpreter_fs_amd import ops as bk  # noqa: E402

bk.init(0)
rng = np.random.default_rng(3)
bad = 0
for n in (1, 127, 128, 1000, 8191, 8192, 65536 + 17, 1 << 20, (1 << 22) + 5, 12_345_679, 50_000_000):
    for dt in (np.float64, np.float32):
        h = rng.standard_normal(n).astype(dt)
        d = bk.asarray(h)
        h64 = h.astype(np.float64)
        ref = {"sum": h64.sum(), "square_sum": np.square(h64).sum(), "max": h64.max(), "min": h64.min()}
        got = {"sum": float(bk.sum(d)), "square_sum": float(bk.square_sum(d)), "max": float(d.max()),
               "min": float(d.min())}
        tol = {"sum": 1e-12 * np.abs(h64).sum(), "square_sum": 1e-12 * ref["square_sum"], "max": 0.0, "min": 0.0}
        for k in ref:
            if not abs(got[k] - ref[k]) <= tol[k]:
                bad += 1
                print("MISMATCH", n, dt.__name__, k, got[k], ref[k])
print("layout", os.environ.get("BK_REDUCE_LAYOUT", "stride"), "mismatches", bad)
sys.exit(1 if bad else 0)
