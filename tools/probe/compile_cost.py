"""What compiling the headline payload costs on this host (the sandbox does it
on every request), against unmarshalling the same code object."""
import marshal
import os
import time

src = open(os.path.join(os.path.dirname(__file__), "..", "..", "examples", "benchmark_numpy_gpu.py")).read()
for _ in range(20):
    compile(src, "/workspace/script.py", "exec", dont_inherit=True)
n = 500
t = time.perf_counter()
for _ in range(n):
    c = compile(src, "/workspace/script.py", "exec", dont_inherit=True)
t1 = time.perf_counter()
blob = marshal.dumps(c)
for _ in range(n):
    marshal.loads(blob)
t2 = time.perf_counter()
print(f"compile {1e6 * (t1 - t) / n:.1f} us, marshal.loads {1e6 * (t2 - t1) / n:.1f} us, {len(src)} B source, {len(blob)} B code")
