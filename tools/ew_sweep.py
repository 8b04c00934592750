"""Grid-size sweep for the streaming kernels (square, Philox, add) on one
MI355X: BK_STREAM_BLOCKS_PER_CU in {4..64}, HIP-event timing, same process."""

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bee_code_interpreter_fs_amd import ops as bk  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    bk.synchronize()
    ts = []
    for _ in range(reps):
        with bk.Timer() as t:
            fn()
        ts.append(t.ms)
    return statistics.median(ts)


def main():
    bk.init()
    n = 10**8
    x = bk.random.rand(n)
    y = bk.random.rand(n)
    for bpc in (4, 8, 16, 32, 64, 128):
        os.environ["BK_STREAM_BLOCKS_PER_CU"] = str(bpc)
        sq = timed(lambda: bk.square(x)._materialize())
        rnd = timed(lambda: bk.random.rand(n))
        add = timed(lambda: x + y)
        print(json.dumps({"blocks_per_cu": bpc, "square_TBps": round(n * 16 / sq / 1e9, 3),
                          "philox_TBps": round(n * 8 / rnd / 1e9, 3), "add_TBps": round(n * 24 / add / 1e9, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
