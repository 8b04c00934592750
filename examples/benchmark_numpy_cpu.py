# The numpy form of the headline workload: 1e8 uniform doubles, squared and
# summed (expected ~1e8/3).  benchmark_numpy_gpu.py runs the same math on the
# MI355X through the beekern HIP kernels.
import time

import numpy as np

t0 = time.time()
x = np.random.rand(100_000_000)
total = np.sum(np.square(x))
print(f"Result: {total}")
print(f"Execution Time: {time.time() - t0:.4f} seconds")
