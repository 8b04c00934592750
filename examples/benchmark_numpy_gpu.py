# benchmark-numpy payload, MI355X edition: the reference's workload
# (examples/benchmark-numpy.py: 1e8 float64 uniform draws, square, sum) on
# the sandbox's pinned GPU through the hand-written beekern kernels, plus the
# 4096^3 bf16 GEMM of BASELINE config 3.  Same printed lines as the original,
# plus the GEMM checksum and a check of every row of the GEMM against an
# independent product:  rowsum(A @ B.T) = A @ colsum(B)
# (row / column sums by the axis-reduction kernel, A @ colsum(B) by the GEMV
# path), so every run checks its own GEMM -- one corrupt 256x256 tile moves
# 256 row sums by ~300 each; bf16 rounding keeps a correct GEMM's rows within
# a few units (bench.py gemm_row_ok).
import time

import beekern as bk


def gpu_intensive_computation():
    n = 10**8
    a = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    b = bk.random.uniform(-1, 1, (4096, 4096), dtype="bfloat16")
    c = bk.matmul(a, b.T)              # MFMA bf16 GEMM, f32 accumulate (queued behind the draws)
    x = bk.random.rand(n)              # Philox4x32-10, f64
    result = bk.sum(bk.square(x))      # fused square+sum (the GPU works the GEMM off meanwhile)
    rows = bk.sum(c, axis=1)           # row sums of C, f64-accumulated
    checksum = bk.sum(rows)
    return result, checksum, a, b, rows


def gemm_row_error(a, b, rows):
    s = bk.sum(b, axis=0).astype("bfloat16").reshape(1, 4096)     # colsum(B) as a 1 x K row
    ref = bk.gemm_bf16_tn(a, s, out_dtype="float32").reshape(4096)  # A @ colsum(B), the GEMV kernel
    return bk.max_abs_diff(rows, ref)


start_time = time.time()
result, checksum, a, b, rows = gpu_intensive_computation()
end_time = time.time()
print("Result:", result)
print("GEMM checksum:", checksum)
print("GEMM max row error:", gemm_row_error(a, b, rows))
print("Execution Time:", end_time - start_time, "seconds")
