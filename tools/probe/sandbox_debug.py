"""What does a minimal GPU sandbox do beyond its zygote?  Runs the headline
payload through a live service (one GPU slot) with BEE_DEBUG_NEW_MODULES=1:
each sandbox reports the modules it imported that its zygote had not, and its
phase stamps; prints them with the per-request timings.

    python tools/probe/sandbox_debug.py [--n 5]
"""

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--payload", default=os.path.join(ROOT, "examples", "benchmark_numpy_gpu.py"))
    ap.add_argument("--cpu", action="store_true", help="no kernel broker (a CPU payload on a host without a GPU)")
    ap.add_argument("--env", action="append", default=[], help="NAME=VALUE for the service (repeatable)")
    args = ap.parse_args()
    for kv in args.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    os.environ["BEE_DEBUG_NEW_MODULES"] = "1"
    os.environ["BEE_DEBUG_BOOT"] = "1"  # the zygote's C bootstrap, per step (lands in the executor log)
    os.environ["BEE_DEBUG_ZYGOTE_MEM"] = "1"  # each zygote's memory rollup (executor log)
    from tests.harness import ServiceHarness, ensure_native_executor

    ensure_native_executor()
    src = open(args.payload).read()
    # (tmpfs, as bench.py: file creation in a disk-backed /tmp costs the
    # bootstrap ~0.25 ms more per sandbox on the MI355X box)
    tmp = tempfile.mkdtemp(prefix="bee-dbg-", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    kw = dict(workers_per_gpu_target=1, min_workers_per_gpu_target=4, light_workers_per_gpu_target=1,
              default_timeout=120.0)
    if args.cpu:
        kw.update(broker_enabled=False, worker_warm_gpu=False, workers_per_gpu_target=0)
    h = ServiceHarness(tmp, gpu_ids=[0], **kw)
    h.start()
    try:
        for i in range(args.n):
            r = h.call(h.ctx.code_executor.execute(source_code=src), timeout=300)
            lines = [l for l in r.stderr.splitlines() if l.startswith(("NEW_MODULES", "STAMPS", "TEARDOWN"))]
            print(json.dumps({"i": i, "exit": r.exit_code, "debug": lines,
                              "timings": {k: round(v, 3) for k, v in sorted(r.timings_ms.items())}}), flush=True)
    finally:
        h.stop()
        import glob

        for log in glob.glob(os.path.join(tmp, "sandboxes", "*", ".run", "executor.log")):
            lines = list(open(log, errors="replace"))
            for l in lines:
                if l.startswith("ZYGOTE_MEM"):  # (and ZYGOTE_MEM_SMALL)
                    print(l.strip())
            boots = [l.strip() for l in lines if l.startswith("BOOT")]
            for l in boots[-args.n:]:
                print(l)
        import shutil

        shutil.rmtree(tmp, ignore_errors=True)  # (/dev/shm is memory)


if __name__ == "__main__":
    main()
