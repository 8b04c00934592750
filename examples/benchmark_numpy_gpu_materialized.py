# benchmark-numpy payload, MI355X edition, materialised draws: the reference's workload
# (examples/benchmark-numpy.py: 1e8 float64 uniform draws, square, sum) on
# the sandbox's pinned GPU through the hand-written beekern kernels, plus the
# 4096^3 bf16 GEMM of BASELINE config 3.  Same printed lines as the original,
# plus the GEMM checksum and its independent reference:
#   sum(A @ B.T) = colsum(A) . colsum(B)
# (column sums by the axis-reduction kernel, dotted in f64), so every run
# checks its own GEMM.
import time

import beekern as bk

bk.set_lazy_random(False)  # materialise every draw in HBM, as numpy does (800 MB for 1e8 f64)


def gpu_intensive_computation():
    n = 10**8
    x = bk.random.rand(n)              # Philox4x32-10, f64, stays in HBM
    result = bk.sum(bk.square(x))      # fused square+sum: one HBM pass
    a = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    b = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    c = bk.matmul(a, b.T)              # MFMA bf16 GEMM, f32 accumulate
    checksum = bk.sum(c)
    return result, checksum, a, b


def gemm_reference(a, b):
    return bk.dot(bk.sum(a, axis=0), bk.sum(b, axis=0))  # column sums, f64-accumulated


start_time = time.time()
result, checksum, a, b = gpu_intensive_computation()
end_time = time.time()
print("Result:", result)
print("GEMM checksum:", checksum)
print("GEMM reference:", gemm_reference(a, b))
print("Execution Time:", end_time - start_time, "seconds")
