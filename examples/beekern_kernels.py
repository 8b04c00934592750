# The preloaded MI355X kernel library, without importing torch: allocations and
# launches go through the executor's kernel broker (light sandbox).
import beekern as bk

rng = bk.random.default_rng(1)
x = rng.random(1 << 24)
print("mean of squares:", float(bk.sum(bk.square(x))) / x.size)
a = rng.uniform(-1, 1, (1024, 1024), dtype="bfloat16")
c = bk.matmul(a, a.T)
print("gemm shape:", c.shape, "checksum:", float(bk.sum(c)))
