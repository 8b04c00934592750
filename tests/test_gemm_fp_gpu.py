"""The f64 / f32 MFMA GEMM (csrc/kernels/gemm_fp.hip) against fp64 numpy.

numpy's own matmul precision is the contract: an f64 product may differ
from the fp64 reference only by the rounding of a blocked dot product
(relative error <= 1e-12 * sqrt(K) of the magnitude scale |A|.|B|), an f32
product by f32 rounding (<= 1e-5).  Every transpose combination is a
``.T`` view read in place; ragged shapes, unaligned leading dimensions,
vectors and NaNs are covered.  Large f32 products run on the bf16 MFMA
through the six-piece split (``bk_gemm_f32x6``) under the same f32 bound;
operands the split cannot represent take the plain f32 kernel, bitwise."""

import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(c, a64, b64, dtype):
    ref = a64 @ b64
    scale = np.abs(a64) @ np.abs(b64)
    err = np.abs(c.astype(np.float64) - ref) / np.maximum(scale, 1e-300)
    K = a64.shape[-1]
    tol = 1e-12 * math.sqrt(K) if dtype == "float64" else 1e-5
    assert float(err.max()) <= tol, (float(err.max()), tol)


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("M,N,K", [(128, 128, 16), (256, 384, 512), (1000, 777, 333), (1, 513, 64), (513, 1, 64),
                                   (64, 64, 1), (129, 127, 17), (2048, 2048, 2048)])
def test_gemm_fp_matches_fp64(gpu, dtype, M, N, K):
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    a_h = rng.standard_normal((M, K)).astype(dtype)
    b_h = rng.standard_normal((K, N)).astype(dtype)
    c = gpu.matmul(gpu.asarray(a_h), gpu.asarray(b_h))
    assert c.dtype == dtype and c.shape == (M, N)
    _check(c.numpy(), a_h.astype(np.float64), b_h.astype(np.float64), dtype)


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("ta,tb", [(True, False), (False, True), (True, True)])
def test_gemm_fp_transposed_views(gpu, dtype, ta, tb):
    """np.dot(a.T, b) and friends: the view's buffer is read in place."""
    M, N, K = 300, 200, 260
    rng = np.random.default_rng(11)
    a_h = rng.standard_normal((K, M) if ta else (M, K)).astype(dtype)
    b_h = rng.standard_normal((N, K) if tb else (K, N)).astype(dtype)
    a, b = gpu.asarray(a_h), gpu.asarray(b_h)
    c = gpu.matmul(a.T if ta else a, b.T if tb else b).numpy()
    a64 = a_h.astype(np.float64)
    b64 = b_h.astype(np.float64)
    _check(c, a64.T if ta else a64, b64.T if tb else b64, dtype)


def test_gemm_fp_unaligned_leading_dimensions(gpu):
    """Leading dimensions that are not a 16-B multiple take the element-load
    path; a sub-matrix of a wider buffer (lda > K) is read in place."""
    from bee_code_interpreter_fs_amd.ops import _native
    from bee_code_interpreter_fs_amd.ops.array import DeviceArray, driver

    M, N, K, lda, ldb, ldc = 131, 67, 45, 47, 69, 71
    rng = np.random.default_rng(5)
    A = rng.standard_normal((M, lda))
    B = rng.standard_normal((K, ldb))
    a, b = gpu.asarray(A), gpu.asarray(B)
    c = DeviceArray((M, ldc), "float64")
    gpu.zeros(1)  # (driver initialised)
    driver().gemm_fp(_native.DTYPE_CODES["float64"], False, False, a.ptr, b.ptr, c.ptr, M, N, K, lda, ldb, ldc)
    _check(c.numpy()[:, :N], A[:, :K], B[:, :N], "float64")


@pytest.mark.parametrize("M,N,K,lda,ldb,ldc", [(130, 126, 34, 34, 126, 126), (70, 2, 18, 24, 4, 5),
                                                (200, 136, 1000, 1002, 140, 137), (1, 64, 2, 2, 64, 64),
                                                (64, 65, 4098, 4100, 66, 65), (3000, 40, 96, 96, 40, 40)])
@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_gemm_fp_ragged_and_padded(gpu, dtype, M, N, K, lda, ldb, ldc):
    """Row-major f64 / f32 on the 16-B load path: ragged M / N / K, K not a
    multiple of the 16-deep tile (its partial tile goes first), sub-matrices
    of wider buffers (lda > K, ldb > N, NaN-filled past the edges) and
    ldc > N, against fp64; the columns past N are left alone, and repeats are
    bitwise the same."""
    from bee_code_interpreter_fs_amd.ops import _native
    from bee_code_interpreter_fs_amd.ops.array import DeviceArray, driver

    rng = np.random.default_rng(M + 3 * N + 7 * K)
    # NaN wherever the product must not read: A's columns past K, B's
    # columns past N and 16 rows past K (a tile read past the edge shows up
    # as NaN in C)
    A = rng.standard_normal((M, lda))
    A[:, K:] = np.nan
    B = rng.standard_normal((K + 16, ldb))
    B[K:, :] = np.nan
    B[:, N:] = np.nan
    A, B = A.astype(dtype), B.astype(dtype)
    a, b = gpu.asarray(A), gpu.asarray(B)
    c = gpu.asarray(np.full((M, ldc), 7.0, dtype=dtype))
    dt = _native.DTYPE_CODES[dtype]
    driver().gemm_fp(dt, False, False, a.ptr, b.ptr, c.ptr, M, N, K, lda, ldb, ldc)
    first = c.numpy()
    assert (first[:, N:] == 7.0).all()
    _check(first[:, :N], A[:, :K].astype(np.float64), B[:K, :N].astype(np.float64), dtype)
    driver().gemm_fp(dt, False, False, a.ptr, b.ptr, c.ptr, M, N, K, lda, ldb, ldc)
    np.testing.assert_array_equal(c.numpy(), first)
    assert isinstance(c, DeviceArray)


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_gemm_fp_wide_leading_dimension_past_31_bit_offsets(gpu, dtype):
    """Rows 256 MiB apart, so row 8 of A starts 2 GiB into the buffer: the
    buffer-descriptor loads (32-bit offsets) must not take the product -- the
    launcher falls back to the guarded loads (gemm_fp.hip, fits()) -- and
    every row still lands in C (a wrapped offset would read another row)."""
    from bee_code_interpreter_fs_amd.ops import _native
    from bee_code_interpreter_fs_amd.ops.array import driver

    M, N, K = 9, 40, 64
    lda = (1 << 28) // np.dtype(dtype).itemsize
    rng = np.random.default_rng(17)
    A = np.zeros((M, lda), dtype=dtype)  # (2.25 GiB; untouched pages stay unmapped on the host)
    A[:, :K] = rng.standard_normal((M, K))
    a_k = A[:, :K].astype(np.float64)
    B = rng.standard_normal((K, N)).astype(dtype)
    a, b = gpu.asarray(A), gpu.asarray(B)
    del A
    c = gpu.asarray(np.zeros((M, N), dtype=dtype))
    driver().gemm_fp(_native.DTYPE_CODES[dtype], False, False, a.ptr, b.ptr, c.ptr, M, N, K, lda, N, N)
    _check(c.numpy(), a_k, B.astype(np.float64), dtype)
    del a


def test_gemm_fp_buffer_loads_on_a_matrix_past_4_gib(gpu):
    """A 4.5 GB f64 operand whose 64-row panels still have 31-bit offsets
    (lda 800000 elements, so the buffer-descriptor loads take it): the
    descriptor's 32-bit range must be capped, not wrapped -- wrapped, the
    range from the first tile's row would end 28 rows in, and the rows past
    it would read as zero."""
    from bee_code_interpreter_fs_amd.ops import _native
    from bee_code_interpreter_fs_amd.ops.array import driver

    M, N, K, lda = 700, 64, 64, 800_000
    rng = np.random.default_rng(19)
    A = np.zeros((M, lda))  # (4.5 GB; untouched pages stay unmapped on the host)
    A[:, :K] = rng.standard_normal((M, K))
    a_k = A[:, :K].copy()
    B = rng.standard_normal((K, N))
    a, b = gpu.asarray(A), gpu.asarray(B)
    del A
    c = gpu.asarray(np.zeros((M, N)))
    driver().gemm_fp(_native.DTYPE_CODES["float64"], False, False, a.ptr, b.ptr, c.ptr, M, N, K, lda, N, N)
    _check(c.numpy(), a_k, B, "float64")
    del a


def test_gemm_fp_propagates_nan_and_inf(gpu):
    a_h = np.ones((128, 64))
    b_h = np.ones((64, 128))
    a_h[3, 5] = np.nan
    b_h[7, 9] = np.inf
    c = gpu.matmul(gpu.asarray(a_h), gpu.asarray(b_h)).numpy()
    want = a_h @ b_h
    np.testing.assert_array_equal(np.isnan(c), np.isnan(want))
    np.testing.assert_array_equal(np.isinf(c), np.isinf(want))


def test_gemm_fp_rejects_bad_arguments(gpu):
    from bee_code_interpreter_fs_amd.ops import _native

    lib = _native.lib()
    assert lib.bk_gemm_fp(2, 0, 0, 8, 8, 8, 4, 4, 4, 4, 4, 4, None) == 1  # bf16 is not this kernel's
    assert lib.bk_gemm_fp(1, 0, 0, 8, 8, 8, 4, 4, 4, 3, 4, 4, None) == 1  # lda < K
    assert lib.bk_gemm_fp(1, 1, 0, 8, 8, 8, 4, 4, 4, 3, 4, 4, None) == 1  # A^T: lda < M
    assert lib.bk_gemm_fp(1, 0, 0, 8, 8, 8, 0, 4, 4, 4, 4, 4, None) == 1  # empty


def test_unmodified_numpy_matmul_under_offload(gpu, monkeypatch):
    """``np.random.rand(n, n) @ np.random.rand(n, n)`` with the offload on:
    the product is the f64 MFMA GEMM, the values numpy's to f64 rounding."""
    from bee_code_interpreter_fs_amd.ops import numpy_offload

    monkeypatch.setattr(numpy_offload, "_GEN", [])
    numpy_offload.patch_numpy_random(np.random, setter=lambda o, k, v: monkeypatch.setattr(o, k, v, raising=False))
    a = np.random.rand(1024, 1024)
    b = np.random.rand(1024, 1024)
    c = a @ b
    assert isinstance(c, numpy_offload.OffloadArray) and c.on_device and c.dtype == np.float64
    g = np.random.default_rng(3).standard_normal((2048, 512))  # 2**20 elements: the offload threshold
    d = np.dot(g.T, g)  # a Generator draw, a .T view read in place
    assert isinstance(d, numpy_offload.OffloadArray) and d.on_device
    a_h, b_h, g_h = np.asarray(a), np.asarray(b), np.asarray(g)
    _check(np.asarray(c), a_h, b_h, "float64")
    _check(np.asarray(d), g_h.T, g_h, "float64")


def _x6(gpu, a_h, b_h, ta, tb, M, N, K):
    """bk_gemm_f32x6 through the driver; a_h / b_h are the stored buffers."""
    from bee_code_interpreter_fs_amd.ops.array import DeviceArray, driver, f32x6_workspace_bytes

    a, b = gpu.asarray(a_h), gpu.asarray(b_h)
    c = DeviceArray((M, N), "float32")
    nbytes = f32x6_workspace_bytes(M, N, K)
    ws = DeviceArray((nbytes // 2,), "bfloat16")
    driver().gemm_f32x6(ta, tb, a.ptr, b.ptr, c.ptr, M, N, K, a_h.shape[1], b_h.shape[1], N, ws.ptr, nbytes)
    return c.numpy()


def _native_f32(gpu, a_h, b_h, ta, tb, M, N, K):
    from bee_code_interpreter_fs_amd.ops.array import DeviceArray, driver

    a, b = gpu.asarray(a_h), gpu.asarray(b_h)
    c = DeviceArray((M, N), "float32")
    driver().gemm_fp(0, ta, tb, a.ptr, b.ptr, c.ptr, M, N, K, a_h.shape[1], b_h.shape[1], N)
    return c.numpy()


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 260), (1000, 777, 333), (129, 1030, 17)])
def test_gemm_f32x6_matches_fp64(gpu, M, N, K, ta, tb):
    """The split product: f32-level error in every orientation, ragged M, N
    and K (the pieces' K blocks are zero-padded to 64)."""
    rng = np.random.default_rng(M + 5 * N + 11 * K + 2 * ta + tb)
    a_h = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    b_h = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    c = _x6(gpu, a_h, b_h, ta, tb, M, N, K)
    a64, b64 = a_h.astype(np.float64), b_h.astype(np.float64)
    _check(c, a64.T if ta else a64, b64.T if tb else b64, "float32")


@pytest.mark.parametrize("bad", [np.inf, -np.inf, np.nan, 3.0e38, 1.0e-35, -2.0e-33])
def test_gemm_f32x6_falls_back_bitwise_outside_the_split_range(gpu, bad):
    """inf / NaN (inf times a zero piece would be NaN), values whose bf16 head
    overflows and values whose pieces leave the normal range: the gated f32
    kernel recomputes C, so the result is the plain f32 kernel's, bitwise."""
    M, N, K = 256, 320, 96
    rng = np.random.default_rng(9)
    a_h = rng.standard_normal((M, K)).astype(np.float32)
    b_h = rng.standard_normal((K, N)).astype(np.float32)
    b_h[17, 33] = bad
    got = _x6(gpu, a_h, b_h, False, False, M, N, K)
    want = _native_f32(gpu, a_h, b_h, False, False, M, N, K)
    np.testing.assert_array_equal(got, want)
    # and back in range, the split runs again (the flag is per call)
    b_h[17, 33] = 0.5
    c = _x6(gpu, a_h, b_h, False, False, M, N, K)
    _check(c, a_h.astype(np.float64), b_h.astype(np.float64), "float32")


def test_large_f32_matmul_routes_to_the_split_and_keeps_f32_precision(gpu):
    """gpu.matmul of a 2048 x 2048 x 1024 f32 product (2^32 multiply-adds)
    takes the split; the error against fp64 stays at f32 rounding level."""
    rng = np.random.default_rng(21)
    a_h = rng.uniform(-1, 1, (2048, 1024)).astype(np.float32)
    b_h = rng.uniform(-1, 1, (1024, 2048)).astype(np.float32)
    c = gpu.matmul(gpu.asarray(a_h), gpu.asarray(b_h)).numpy()
    a64, b64 = a_h.astype(np.float64), b_h.astype(np.float64)
    err = np.abs(c - a64 @ b64) / (np.abs(a64) @ np.abs(b64))
    assert float(err.max()) < 2e-6, float(err.max())


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_gemm_fp_split_k_is_deterministic_and_keeps_c_gaps(gpu, dtype):
    """Small products split K over two wave groups of one workgroup (group 1
    hands its half to group 0 through LDS): the result is bitwise the same on
    every repeat, within the dtype's bound, and a C with ldc > N keeps the
    columns past N untouched (no memset of C)."""
    from bee_code_interpreter_fs_amd.ops import _native
    from bee_code_interpreter_fs_amd.ops.array import DeviceArray, driver

    M, N, K, ldc = 200, 136, 1024, 150
    rng = np.random.default_rng(17)
    A = rng.standard_normal((M, K)).astype(dtype)
    B = rng.standard_normal((K, N)).astype(dtype)
    a, b = gpu.asarray(A), gpu.asarray(B)
    c = gpu.asarray(np.full((M, ldc), 7.0, dtype=dtype))
    dt = _native.DTYPE_CODES[dtype]
    driver().gemm_fp(dt, False, False, a.ptr, b.ptr, c.ptr, M, N, K, K, N, ldc)
    first = c.numpy()
    assert (first[:, N:] == 7.0).all()
    _check(first[:, :N], A.astype(np.float64), B.astype(np.float64), dtype)
    for _ in range(3):
        driver().gemm_fp(dt, False, False, a.ptr, b.ptr, c.ptr, M, N, K, K, N, ldc)
        np.testing.assert_array_equal(c.numpy(), first)
    big = gpu.matmul(gpu.asarray(rng.standard_normal((1024, 1024)).astype(dtype)),
                     gpu.asarray(rng.standard_normal((1024, 1024)).astype(dtype)))
    assert isinstance(big, DeviceArray)
