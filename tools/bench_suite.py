"""All BASELINE.json configs on this node, one JSON line each (1 GPU box):

  1. hello_world on a CPU-only executor                  (--cpu-only)
  2. benchmark-fib on 1 GPU-pinned executor
  3. benchmark-numpy via HIP kernels on 1 GPU (headline)  + the unmodified
     numpy payload on CPU in the same pod, and under the numpy offload;
     likewise an unmodified numpy 4096^3 f64 matmul script
  4./5. (8 GPUs: 64 concurrent Executes, gang all-reduce) are the driver's
     N=8 bench.py run; on the 1-GPU box they are skipped.

    python tools/bench_suite.py --out gpurun_out/suite.jsonl
"""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RUNS = [
    ("hello_cpu", ["--workload", "hello", "--cpu-only", "--steps", "50"]),
    ("hello_gpu_pod", ["--workload", "hello", "--steps", "50"]),
    ("fib_gpu_pod", ["--workload", "fib", "--steps", "4", "--concurrency", "16"]),
    ("numpy_gpu", ["--workload", "numpy_gpu", "--steps", "30"]),
    ("numpy_cpu", ["--workload", "numpy_cpu", "--steps", "3", "--concurrency", "4"]),
    # the same unmodified payload with the opt-in numpy offload (ops/numpy_offload.py)
    ("numpy_cpu_offload", ["--workload", "numpy_cpu", "--numpy-offload", "--steps", "30"]),
    ("scientific_gpu_pod", ["--workload", "scientific", "--steps", "30"]),
    # unmodified numpy np.random.rand(4096, 4096) @ np.random.rand(4096, 4096)
    # (examples/numpy_matmul_4096.py): OpenBLAS on the sandbox's CPUs, then
    # the same script under the offload (the f64 MFMA GEMM)
    ("numpy_matmul_cpu", ["--workload", "numpy_cpu", "--payload", "examples/numpy_matmul_4096.py", "--steps", "2",
                          "--concurrency", "2"]),
    ("numpy_matmul_offload", ["--workload", "numpy_cpu", "--payload", "examples/numpy_matmul_4096.py",
                              "--numpy-offload", "--steps", "10"]),
]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "bench_suite.jsonl"))
    p.add_argument("--only", nargs="*")
    p.add_argument("--timeout", type=int, default=300)
    a = p.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    rc = 0
    with open(a.out, "a") as out:
        for name, extra in RUNS:
            if a.only and name not in a.only:
                continue
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--warmup", "2", *extra]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=ROOT)
            except subprocess.TimeoutExpired:
                print(json.dumps({"run": name, "error": "timeout"}), flush=True)
                rc = 124
                break  # stop: the box may be in a bad state
            line = next((l for l in reversed(r.stdout.splitlines()) if l.startswith("{")), None)
            rec = {"run": name, **(json.loads(line) if line else {"error": r.stderr[-800:], "rc": r.returncode})}
            out.write(json.dumps(rec) + "\n")
            out.flush()
            print(json.dumps({k: rec.get(k) for k in ("run", "value", "p50_latency_ms", "p95_latency_ms", "errors")}), flush=True)
            if r.returncode != 0:
                rc = r.returncode
                if r.returncode < 0 or r.returncode >= 124:
                    break
    sys.exit(rc)


if __name__ == "__main__":
    main()
