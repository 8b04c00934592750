# Unmodified numpy: the product of two 4096 x 4096 uniform f64 draws (the
# review's round-5 ask: `np.random.rand(4096, 4096) @ np.random.rand(4096,
# 4096)`), checked two ways.  On the CPU this is OpenBLAS dgemm; under
# Execute(numpy_offload=True) the draws are device arrays and `@` runs the
# f64 MFMA GEMM (csrc/kernels/gemm_fp.hip) at numpy's precision.
import numpy as np

a = np.random.rand(4096, 4096)
b = np.random.rand(4096, 4096)
c = a @ b
# the grand mean of c is 4096 / 4 = 1024 (its sd over draws is ~0.2)
m = float(c.mean())
# every row of c against an independent product: rowsum(a @ b) = a @ rowsum(b)
rows = np.asarray(c.sum(axis=1))
ref = np.asarray(a @ np.asarray(b.sum(axis=1)))
rel = float(np.max(np.abs(rows - ref) / np.abs(ref)))
print("mean:", m, "max row rel err:", rel)
assert abs(m - 1024.0) < 2.0, m
assert rel < 1e-9, rel
