"""Grid sweep of the materialised payload's two HBM-bound kernels on one
MI355X: the f64 square-sum over 1e8 values (bk_reduce kRedSquareSum, 800 MB
read) across BK_REDUCE_BLOCKS, and the f64 Philox store (800 MB written) for reference.  The knob is read
once per process, so every point runs in a child process.

    python tools/reduce_sweep.py [--n 100000000] [--reps 30]

One JSON line per point: median / min device time (HIP events) and TB/s.
"""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, statistics, sys
sys.path.insert(0, {root!r})
from bee_code_interpreter_fs_amd import ops as bk
bk.init(0)
n, reps, what = {n}, {reps}, {what!r}
bk.set_lazy_random(False)
x = bk.random.default_rng(1).random(n)   # materialised f64
if what in ("torch_sum", "d2d_copy"):
    import torch
    tx = torch.rand(n, dtype=torch.float64, device="cuda")
    ty = torch.empty_like(tx)
def once():
    if what == "square_sum":
        return bk.square_sum(x)
    if what == "torch_sum":
        return tx.sum()
    if what == "d2d_copy":
        return ty.copy_(tx)
    sys.modules["bee_code_interpreter_fs_amd.ops.array"].driver().rand(0, x.ptr, n, x.code, 7, 0, 0.0, 1.0)
for _ in range(3):
    once()
bk.synchronize()
ts = []
for _ in range(reps):
    if what in ("torch_sum", "d2d_copy"):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); once(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
        continue
    with bk.Timer() as t:
        once()
    ts.append(t.ms)
med = statistics.median(ts)
print(json.dumps({{"what": what, "median_us": round(med * 1e3, 2), "min_us": round(min(ts) * 1e3, 2),
                  "TBps_median": round(n * 8 / (med * 1e-3) / 1e12, 3)}}))
"""


def run(what, env_extra, n, reps):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, n=n, reps=reps, what=what)], env=env,
                       capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    out = json.loads(line[-1]) if line else {"what": what, "error": p.stderr[-500:]}
    out.update(env_extra)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10**8)
    ap.add_argument("--reps", type=int, default=30)
    # reduce.hip reduce_1pass (stride) / reduce_chunked (chunk) / reduce_ldsdma (ldsdma)
    ap.add_argument("--layouts", default="stride,chunk")
    ap.add_argument("--blocks", default="384,512,640,768,1024")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--unrolls", default="16", help="BK_REDUCE_UNROLL values (grid-stride layout: 4 / 8 / 16)")
    ap.add_argument("--no-refs", action="store_true", help="skip the Philox store / torch / copy reference rows")
    a = ap.parse_args()
    for _ in range(a.rounds):  # interleaved repeats: box-to-box and run-to-run noise is a few %
        for layout in a.layouts.split(","):
            for blocks in a.blocks.split(","):
                for u in (a.unrolls.split(",") if layout == "stride" else ["16"]):
                    env = {"BK_REDUCE_BLOCKS": blocks, "BK_REDUCE_LAYOUT": layout}
                    if u != "16":
                        env["BK_REDUCE_UNROLL"] = u
                    run("square_sum", env, a.n, a.reps)
    if a.no_refs:
        return
    run("philox_store", {}, a.n, a.reps)
    run("torch_sum", {}, a.n, a.reps)   # torch's own reduction over the same 800 MB (read roofline reference)
    run("d2d_copy", {}, a.n, a.reps)    # hipMemcpy device-to-device: 800 MB read + 800 MB written  # (its grid is fixed: kDrawBlocksPerCU, profiles/archive/r3_philox_grid_sweep.log)


if __name__ == "__main__":
    main()
