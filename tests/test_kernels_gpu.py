"""Numerics of the hand-written HIP kernels vs plain fp32/fp64 references.

Run on an MI355X: ``python -m pytest tests -m gpu``.  Each kernel is checked
against numpy / torch computed in fp32 (bf16 inputs) or fp64.
"""

import os

import numpy as np
import pytest

from .gemm_check import assert_gemm_close, gemm_error

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_library_is_native(gpu):
    from bee_code_interpreter_fs_amd.ops import _native

    assert _native.is_loaded()
    info = gpu.device_info()
    assert info["arch"].startswith("gfx950"), info
    assert info["compute_units"] >= 256


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("n", [1, 7, 1000, 1 << 20, 10_000_019])
def test_uniform_range_and_moments(gpu, dtype, n):
    x = gpu.random.default_rng(1234).random(n, dtype=dtype)
    h = x.numpy()
    assert h.shape == (n,) and h.dtype == np.dtype(dtype)
    assert (h >= 0).all() and (h < 1).all()
    if n >= 1 << 20:
        assert abs(h.mean() - 0.5) < 2e-3
        assert abs(h.var() - 1 / 12) < 2e-3
    # counter-based: same seed -> same stream, independent of call grouping
    y = gpu.random.default_rng(1234).random(n, dtype=dtype).numpy()
    np.testing.assert_array_equal(h, y)


@pytest.mark.parametrize("n", [1, 7, 4099, 1 << 20])
def test_uniform_streams_match_host_philox_bitwise(gpu, n):
    """Every element of the f64 / f32 U[0,1) streams equals the host
    Philox4x32-10 reference (tests/philox_ref.py, checked against the
    Random123 known-answer vectors), including after an offset advance.
    Scaled draws (lo + span*u) are one fused multiply-add on the GPU, so
    they are held to one rounding of the unfused host expression."""
    from .philox_ref import uniform_f32, uniform_f64

    seed = 0x1234_5678_9ABC_DEF0
    g = gpu.random.default_rng(seed)
    np.testing.assert_array_equal(g.random(n).numpy(), uniform_f64(n, seed))
    off = (n + 1) // 2  # the generator's counter advance for that draw
    np.testing.assert_array_equal(g.random(n).numpy(), uniform_f64(n, seed, off))
    np.testing.assert_array_equal(gpu.random.default_rng(seed).random(n, dtype="float32").numpy(), uniform_f32(n, seed))
    # one rounding of the product apart: 1 ulp at the magnitude of span*u
    # (more ulps of a result that cancels towards 0)
    np.testing.assert_allclose(gpu.random.default_rng(seed).uniform(-2.0, 3.0, n).numpy(),
                               uniform_f64(n, seed, 0, -2.0, 3.0), rtol=0, atol=float(np.spacing(5.0)))
    np.testing.assert_allclose(gpu.random.default_rng(seed).uniform(-1, 1, n, dtype="float32").numpy(),
                               uniform_f32(n, seed, 0, -1.0, 1.0), rtol=0, atol=float(np.spacing(np.float32(2.0))))


@pytest.mark.parametrize("n", [2 * 2 * 16384 * 256 + 12345, 40_000_003])
def test_large_uniform_f64_windows_match_host_philox(gpu, n):
    """Draws long enough for the f64 kernel's two-counters-per-lane loop
    (the 40M draw's 20M pairs exceed one grid stride of 65536 x 256), its
    one-counter tail, the odd last element, and (40M: 320 MB) the
    non-temporal store path: windows at the start, across 4M-pair
    boundaries and at the end equal the host reference stream bit for bit
    (uniform_f64's offset is in pairs)."""
    from .philox_ref import uniform_f64

    seed = 0x0DDB_A11_5EED
    x = gpu.random.default_rng(seed).random(n).numpy()
    stride = 16384 * 256
    w = 4096
    pairs = (n + 1) // 2
    for pair0 in [0, stride - w // 4, 2 * stride - w // 4, 3 * stride - w // 4, 4 * stride - w // 4, pairs - w // 2]:
        if pair0 >= pairs:
            continue
        i0 = 2 * pair0
        m = min(w, n - i0)
        np.testing.assert_array_equal(x[i0:i0 + m], uniform_f64(m, seed, pair0), err_msg=f"window at {i0}")


def test_fused_rand_square_sum_matches_host_reference(gpu):
    """The headline payload's lowering -- sum(square(rand(n))) as one fused
    Philox->square->reduce kernel -- against an fp64 host sum of the
    reference stream."""
    from .philox_ref import uniform_f64

    n = 3_000_001
    got = float(gpu.sum(gpu.square(gpu.random.default_rng(99).random(n))))
    ref = float(np.square(uniform_f64(n, 99)).sum())
    assert abs(got - ref) <= 1e-9 * abs(ref)


def test_uniform_offsets_do_not_overlap(gpu):
    g = gpu.random.default_rng(7)
    a = g.random(1000).numpy()
    b = g.random(1000).numpy()
    assert not np.array_equal(a, b)
    c = gpu.random.default_rng(7).random(2000).numpy()
    np.testing.assert_array_equal(np.concatenate([a, b]), c)


def test_normal_moments(gpu):
    x = gpu.random.default_rng(3).normal(2.0, 3.0, 1 << 22, dtype="float32").numpy()
    assert abs(x.mean() - 2.0) < 0.02 and abs(x.std() - 3.0) < 0.02
    y = gpu.random.default_rng(3).normal(0.0, 1.0, 1 << 21, dtype="float64").numpy()
    assert abs(y.mean()) < 0.01 and abs(y.std() - 1.0) < 0.01


@pytest.mark.parametrize("dtype", ["float64", "float32", "bfloat16"])
@pytest.mark.parametrize("n", [1, 33, 4097, 3_000_001])
def test_unary_ops(gpu, dtype, n):
    rng = np.random.default_rng(0)
    h = rng.uniform(0.1, 2.0, n).astype(np.float64 if dtype == "float64" else np.float32)
    x = gpu.asarray(h, dtype=dtype)
    ref_in = x.numpy().astype(np.float64)
    tol = {"float64": 1e-12, "float32": 2e-6, "bfloat16": 1e-2}[dtype]
    for name, ref in [("sqrt", np.sqrt), ("exp", np.exp), ("log", np.log), ("abs", np.abs), ("tanh", np.tanh)]:
        out = getattr(gpu, name)(x).numpy().astype(np.float64)
        np.testing.assert_allclose(out, ref(ref_in), rtol=tol * 4, atol=tol, err_msg=name)
    sq = gpu.square(x).numpy().astype(np.float64)  # lazy -> materialised
    np.testing.assert_allclose(sq, ref_in * ref_in, rtol=tol * 4, atol=tol)


@pytest.mark.parametrize("dtype", ["float64", "float32", "bfloat16"])
def test_binary_ops(gpu, dtype):
    rng = np.random.default_rng(1)
    a_h, b_h = rng.uniform(0.5, 2, 100_003), rng.uniform(0.5, 2, 100_003)
    a, b = gpu.asarray(a_h, dtype=dtype), gpu.asarray(b_h, dtype=dtype)
    ra, rb = a.numpy().astype(np.float64), b.numpy().astype(np.float64)
    tol = {"float64": 1e-12, "float32": 2e-6, "bfloat16": 1e-2}[dtype]
    for got, ref in [
        (a + b, ra + rb),
        (a - b, ra - rb),
        (a * b, ra * rb),
        (a / b, ra / rb),
        (a * 3.0, ra * 3.0),
        (2.0 - a, 2.0 - ra),
        (1.0 / a, 1.0 / ra),
        (gpu.maximum(a, b), np.maximum(ra, rb)),
    ]:
        np.testing.assert_allclose(got.numpy().astype(np.float64), ref, rtol=tol * 4, atol=tol)


@pytest.mark.parametrize("dtype", ["float64", "float32", "bfloat16"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1 << 16, 12_345_679])
def test_reductions(gpu, dtype, n):
    rng = np.random.default_rng(n)
    h = rng.standard_normal(n)
    x = gpu.asarray(h, dtype=dtype)
    r = x.numpy().astype(np.float64)
    rtol = 1e-10 if dtype == "float64" else 1e-6
    scale = np.abs(r).sum() + 1e-30
    assert abs(gpu.sum(x) - r.sum()) <= rtol * scale
    assert abs(gpu.square_sum(x) - (r * r).sum()) <= rtol * (r * r).sum()
    assert abs(gpu.sum(gpu.square(x)) - (r * r).sum()) <= rtol * (r * r).sum()  # fused path
    assert gpu.amax(x) == r.max() and gpu.amin(x) == r.min()
    y = gpu.asarray(rng.standard_normal(n), dtype=dtype)
    ry = y.numpy().astype(np.float64)
    assert abs(gpu.dot(x, y) - (r * ry).sum()) <= rtol * (np.abs(r * ry).sum() + 1e-30)


def test_reductions_long_array_all_loops(gpu):
    """~1e8 f64 (805 MB, the materialised payload's size): on the capped grid
    (8192 x 256 lanes) each lane takes ~24 vectors -- the 16-in-flight loop,
    two 4-in-flight groups and the one-at-a-time tail all run; the odd
    length leaves a scalar remainder."""
    n = (1 << 26) + (1 << 25) + 12345
    h = np.random.default_rng(11).random(n)
    x = gpu.asarray(h)
    assert abs(float(gpu.sum(x)) - h.sum()) <= 1e-12 * h.sum()
    assert abs(float(gpu.square_sum(x)) - np.dot(h, h)) <= 1e-12 * np.dot(h, h)
    assert float(gpu.amax(x)) == h.max()


def test_reduction_is_deterministic(gpu):
    x = gpu.random.default_rng(5).random(10_000_000)
    vals = {float(gpu.sum(x)) for _ in range(5)}
    assert len(vals) == 1


def test_benchmark_numpy_payload(gpu):
    """benchmark-numpy.py semantics: E[sum(U^2)] = n/3."""
    n = 10**8
    x = gpu.random.rand(n)
    s = gpu.sum(gpu.square(x))
    assert abs(s - n / 3) < 5 * np.sqrt(n * 4 / 45)


def _bf16_round(a):
    import torch

    return torch.from_numpy(a).to(torch.bfloat16).to(torch.float32).numpy()


@pytest.mark.parametrize(
    "m,n,k",
    [(128, 128, 64), (256, 384, 512), (1024, 1024, 1024), (100, 70, 33), (129, 257, 65), (4096, 4096, 4096)],
)
@pytest.mark.parametrize("out_dtype", ["float32", "bfloat16"])
def test_gemm_bf16(gpu, m, n, k, out_dtype):
    rng = np.random.default_rng(m * 7 + n * 3 + k)
    a_h = _bf16_round(rng.uniform(-1, 1, (m, k)).astype(np.float32))
    b_h = _bf16_round(rng.uniform(-1, 1, (k, n)).astype(np.float32))
    a, b = gpu.asarray(a_h, "bfloat16"), gpu.asarray(b_h, "bfloat16")
    c = gpu.matmul(a, b, out_dtype=out_dtype).numpy().astype(np.float64)
    assert_gemm_close(c, a_h, b_h, out_dtype)


def test_gemm_asymmetric_identity(gpu):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 256
    b_h = _bf16_round(np.arange(n * n, dtype=np.float32).reshape(n, n) % 97 / 97.0)
    eye = gpu.asarray(np.eye(n, dtype=np.float32), "bfloat16")
    c = gpu.matmul(eye, gpu.asarray(b_h, "bfloat16"), out_dtype="float32").numpy()
    np.testing.assert_array_equal(c, b_h)
    ct = gpu.matmul(gpu.asarray(b_h, "bfloat16"), eye, out_dtype="float32").numpy()
    np.testing.assert_array_equal(ct, b_h)


@pytest.mark.parametrize("out", ["float32", "bfloat16"])
@pytest.mark.parametrize("shape", [(1024, 1024, 1024), (4096, 4096, 4096), (512, 768, 320)])
def test_gemm_bound_catches_a_missing_k_tile(gpu, shape, out):
    """The bound of tests/gemm_check.py is tight enough to matter: the same
    kernel run one 64-deep K tile short of the operands fails it, the full
    product passes (VERDICT r5 "next" #6)."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M, N, K = shape
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    dt = torch.float32 if out == "float32" else torch.bfloat16
    lib = _native.lib()
    s = torch.cuda.current_stream().cuda_stream
    odt = 0 if out == "float32" else 2
    full = torch.zeros(M, N, device="cuda", dtype=dt)
    short = torch.zeros(M, N, device="cuda", dtype=dt)
    assert lib.bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), full.data_ptr(), M, N, K, K, K, N, 1.0, 0.0, odt,
                                       0, s) == 0
    assert lib.bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), short.data_ptr(), M, N, K - 64, K, K, N, 1.0, 0.0,
                                       odt, 0, s) == 0
    torch.cuda.synchronize()
    assert gemm_error(full, a, bt.T, out) <= 1.0
    assert gemm_error(short, a, bt.T, out) > 10.0  # not a near miss


def test_gemm_transposed_view_operand(gpu):
    rng = np.random.default_rng(11)
    a_h = _bf16_round(rng.uniform(-1, 1, (256, 512)).astype(np.float32))
    bt_h = _bf16_round(rng.uniform(-1, 1, (384, 512)).astype(np.float32))
    a, bt = gpu.asarray(a_h, "bfloat16"), gpu.asarray(bt_h, "bfloat16")
    c = gpu.matmul(a, bt.T, out_dtype="float32").numpy()
    assert_gemm_close(c, a_h, bt_h.T)


@pytest.mark.parametrize("rows,cols,ld_in,ld_out", [
    (8, 8, 8, 8), (64, 256, 256, 64), (136, 200, 200, 136), (72, 520, 528, 80),  # 16-B vector path
    (7, 13, 13, 7), (65, 130, 131, 65),                                            # tiled fallback
])
def test_transpose_bf16_bitwise(gpu, rows, cols, ld_in, ld_out):
    """Both transpose kernels (8x8 register blocks for 8-aligned shapes, LDS
    tiles otherwise) against numpy, bit for bit, with padded leading
    dimensions whose padding must stay untouched."""
    from bee_code_interpreter_fs_amd.ops.array import driver

    rng = np.random.default_rng(rows * 1000 + cols)
    src_h = rng.integers(0, 1 << 16, size=(rows, ld_in), dtype=np.uint16)
    sentinel = np.full((cols, ld_out), 0xBEEF, dtype=np.uint16)
    src, dst = gpu.empty((rows * ld_in,), "bfloat16"), gpu.empty((cols * ld_out,), "bfloat16")
    driver().h2d(src.ptr, src_h)
    driver().h2d(dst.ptr, sentinel)
    driver().transpose(src.ptr, dst.ptr, rows, cols, ld_in, ld_out)
    out = np.empty((cols, ld_out), dtype=np.uint16)
    driver().d2h(dst.ptr, out)
    np.testing.assert_array_equal(out[:, :rows], src_h[:, :cols].T)
    np.testing.assert_array_equal(out[:, rows:], sentinel[:, rows:])


@pytest.mark.parametrize("src_dtype", ["float32", "float64"])
@pytest.mark.parametrize("rows,cols,ld_in,ld_out", [(8, 8, 8, 8), (136, 200, 200, 136), (72, 520, 528, 80)])
def test_transpose_to_bf16_bitwise(gpu, src_dtype, rows, cols, ld_in, ld_out):
    """Fused f32/f64 -> bf16 transpose == cast kernel then transpose, bit for
    bit (same rounding: (float) then RNE), padding untouched."""
    from bee_code_interpreter_fs_amd.ops._native import DTYPE_CODES
    from bee_code_interpreter_fs_amd.ops.array import driver

    rng = np.random.default_rng(rows + cols)
    src_h = rng.standard_normal((rows, ld_in)).astype(src_dtype)
    src_h[0, 0], src_h[-1, cols - 1] = 3e38, -0.0  # near the top of the bf16 range; signed zero
    src = gpu.empty((rows * ld_in,), src_dtype)
    driver().h2d(src.ptr, src_h)
    dst = gpu.empty((cols * ld_out,), "bfloat16")
    driver().h2d(dst.ptr, np.full((cols, ld_out), 0xBEEF, dtype=np.uint16))
    driver().transpose(src.ptr, dst.ptr, rows, cols, ld_in, ld_out, DTYPE_CODES[src_dtype])
    fused = np.empty((cols, ld_out), dtype=np.uint16)
    driver().d2h(dst.ptr, fused)
    # two-pass reference on the device: the cast kernel, then the bf16 transpose
    cast = gpu.empty((rows * ld_in,), "bfloat16")
    driver().cast(DTYPE_CODES[src_dtype], DTYPE_CODES["bfloat16"], src.ptr, cast.ptr, rows * ld_in)
    two = gpu.empty((cols * ld_out,), "bfloat16")
    driver().transpose(cast.ptr, two.ptr, rows, cols, ld_in, ld_out)
    ref = np.empty((cols, ld_out), dtype=np.uint16)
    driver().d2h(two.ptr, ref)
    np.testing.assert_array_equal(fused[:, :rows], ref[:, :rows])
    np.testing.assert_array_equal(fused[:, rows:], 0xBEEF)
    # and against the host rounding of the f32 value
    host = _f32_to_bf16_host(src_h[:, :cols].astype(np.float32)).T
    np.testing.assert_array_equal(fused[:, :rows], host)


def _f32_to_bf16_host(a):
    from bee_code_interpreter_fs_amd.ops.array import _f32_to_bf16_bits

    return _f32_to_bf16_bits(a)


@pytest.mark.parametrize("dtype", ["float32", "float64", "bfloat16"])
@pytest.mark.parametrize("shape", [(8, 8), (64, 256), (136, 200), (7, 13), (65, 130)])
def test_transposed_view_materialises_on_device_bitwise(gpu, dtype, shape):
    """DeviceArray.T of f32/f64 arrays: the 4-/8-byte register-block kernel
    (8-aligned shapes) or the scalar fallback, bit for bit."""
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    h = rng.standard_normal(shape).astype(np.float32 if dtype != "float64" else np.float64)
    x = gpu.asarray(h, dtype)
    ref = x.numpy().T
    got = x.T.numpy()
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)


def test_transpose_to_bf16_rejects_unaligned_wide_input(gpu):
    from bee_code_interpreter_fs_amd.ops import _native

    x = gpu.empty((12 * 12,), "float32")
    y = gpu.empty((12 * 12,), "bfloat16")
    assert _native.lib().bk_transpose_to_bf16(0, x.ptr, y.ptr, 12, 12, 12, 12, None) != 0


@pytest.mark.parametrize("b_kind", ["float64", "float32", "float32_T"])
def test_matmul_wide_b_operand(gpu, b_kind):
    """matmul with an f64/f32 row-major b (fused convert+transpose) and with
    an f32 b.T view (conversion only) against fp64."""
    rng = np.random.default_rng(9)
    a_h = _bf16_round(rng.uniform(-1, 1, (512, 256)).astype(np.float32))
    b_h = _bf16_round(rng.uniform(-1, 1, (256, 768)).astype(np.float32))
    if b_kind == "float32_T":
        b = gpu.asarray(np.ascontiguousarray(b_h.T), "float32").T
    else:
        b = gpu.asarray(b_h, b_kind)
    c = gpu.matmul(gpu.asarray(a_h, "bfloat16"), b, out_dtype="float32").numpy()
    assert_gemm_close(c, a_h, b_h)


def test_matmul_row_major_b_large(gpu):
    """bk.matmul(a, b) with a plain row-major b (transpose + TN GEMM) on a
    shape that takes the vectorised transpose and the 256^2 GEMM."""
    rng = np.random.default_rng(5)
    a_h = _bf16_round(rng.uniform(-1, 1, (2048, 1024)).astype(np.float32))
    b_h = _bf16_round(rng.uniform(-1, 1, (1024, 4096)).astype(np.float32))
    c = gpu.matmul(gpu.asarray(a_h, "bfloat16"), gpu.asarray(b_h, "bfloat16"), out_dtype="float32").numpy()
    assert_gemm_close(c, a_h, b_h)


def test_quota_enforced(gpu):
    from bee_code_interpreter_fs_amd.ops import QuotaExceeded

    before = gpu.memory_stats()
    gpu.set_quota(before["in_use"] + (64 << 20))
    try:
        keep = gpu.empty((1 << 20,), "float64")  # 8 MiB fits
        with pytest.raises(QuotaExceeded):
            gpu.empty((16 << 20,), "float64")  # 128 MiB does not
        del keep
    finally:
        gpu.set_quota(0)


def test_torch_interop(gpu):
    import torch

    t = torch.arange(1000, dtype=torch.float32, device="cuda")
    v = gpu.from_torch(t)
    assert float(gpu.sum(v)) == pytest.approx(float(t.sum().item()))
    back = gpu.to_torch(gpu.square(v))
    torch.testing.assert_close(back, t * t)


@pytest.mark.parametrize("shape", [(1000, 1000, 1000), (511, 769, 328), (4095, 4097, 4096), (130, 1, 8)])
@pytest.mark.parametrize("out", ["float32", "bfloat16"])
def test_gemm_edge_kernel_unaligned_shapes(gpu, shape, out):
    """The MFMA edge kernel (variant 6, what `auto` picks for non-tile
    shapes with K % 8 == 0): zero-filled buffer loads past M / N / K, masked
    stores -- against fp64, beta epilogue included, C's padding untouched."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M, N, K = shape
    ldc = N + 8
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    dt = torch.float32 if out == "float32" else torch.bfloat16
    c0 = torch.empty(M, ldc, device="cuda", dtype=dt).uniform_(-1, 1, generator=g)
    c = c0.clone()
    lib = _native.lib()
    # N <= 16: the skinny GEMV kernel (8); K % 64 == 0 and enough 256^2 tiles: the 4-wave kernel's edge
    # mode (7); else the 128^2 edge kernel (6)
    want = 8 if N <= 16 else 7 if ((M + 255) // 256) * ((N + 255) // 256) >= 128 else 6
    assert lib.bk_gemm_bf16_pick(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, ldc,
                                 0 if out == "float32" else 2) == want
    rc = lib.bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, ldc, 0.75, 0.5,
                                     0 if out == "float32" else 2, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert_gemm_close(c[:, :N], a, bt.T, out, alpha=0.75, beta=0.5, c0=c0[:, :N])
    assert torch.equal(c[:, N:], c0[:, N:])  # masked stores: the padding columns are intact


def test_gemm_huge_leading_dimension(gpu):
    """lda > 4.4M: the 4-wave kernel's 32-bit buffer offsets would wrap; the
    dispatcher must route such operands to 64-bit addressing (round-1
    review, weak #3).  A is a 256 x 256 window of rows 4.5M elements apart."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M = N = 256
    K = 256
    lda = 4_500_000
    g = torch.Generator(device="cuda").manual_seed(5)
    store = torch.empty(M * lda, device="cuda", dtype=torch.bfloat16)  # 2.3 GB
    a = store.view(M, lda)[:, :K]
    a.uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    ref = a.double() @ bt.double().T
    lib = _native.lib()
    for variant in (0, 3, 5):
        c = torch.zeros(M, N, device="cuda", dtype=torch.float32)
        rc = lib.bk_gemm_bf16_tn_variant(store.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, lda, K, N, 1.0, 0.0, 0,
                                         variant, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, variant
        torch.cuda.synchronize()
        assert gemm_error(c, a, bt.T) <= 1.0, variant
    del store


@pytest.mark.parametrize("shape", [(257, 300, 64), (4095, 4097, 4096), (600, 256, 512), (256, 1000, 128), (1, 1, 64),
                                   (4000, 4000, 4000), (300, 520, 72), (513, 260, 8), (1100, 1030, 136)])
@pytest.mark.parametrize("out", ["float32", "bfloat16"])
@pytest.mark.parametrize("c_offset", [0, 1])
def test_gemm_256_edge_mode(gpu, shape, out, c_offset):
    """The 4-wave 256^2 kernel in edge mode (variant 7): operand panels
    bounded by the rows that exist, masked element stores on the ragged
    border and wherever C / ldc break 16-B alignment (odd ldc, C offset by
    one element) -- against fp64, beta epilogue, padding intact."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M, N, K = shape
    ldc = N + 3  # odd: no vector store is ever aligned
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + c_offset)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    dt = torch.float32 if out == "float32" else torch.bfloat16
    store0 = torch.empty(M * ldc + 8, device="cuda", dtype=dt).uniform_(-1, 1, generator=g)
    store = store0.clone()
    c = store[c_offset : c_offset + M * ldc].view(M, ldc)
    c0 = store0[c_offset : c_offset + M * ldc].view(M, ldc)
    rc = _native.lib().bk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, ldc, 0.75,
                                               0.5, 0 if out == "float32" else 2, 7,
                                               torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert_gemm_close(c[:, :N], a, bt.T, out, alpha=0.75, beta=0.5, c0=c0[:, :N])
    assert torch.equal(c[:, N:], c0[:, N:])
    assert torch.equal(store[:c_offset], store0[:c_offset]) and torch.equal(store[c_offset + M * ldc:],
                                                                          store0[c_offset + M * ldc:])


def test_gemm_256_edge_mode_refuses_k_not_multiple_of_8(gpu):
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    a = torch.zeros(300, 100, device="cuda", dtype=torch.bfloat16)
    c = torch.zeros(300, 300, device="cuda", dtype=torch.float32)
    rc = _native.lib().bk_gemm_bf16_tn_variant(a.data_ptr(), a.data_ptr(), c.data_ptr(), 300, 300, 99, 100, 100, 300,
                                               1.0, 0.0, 0, 7, torch.cuda.current_stream().cuda_stream)
    assert rc == 1  # kBadArgument: 16-B chunks need K % 8 == 0 (the generic kernel's case)


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("out", ["float32", "bfloat16"])
def test_gemm_kernel_variants_with_beta(gpu, variant, out):
    """Every GEMM kernel (generic / 128^2 / 256^2 by shape / 256^2 8-wave
    phase-pipelined / 256^2 4-wave inline-asm MFMA) against an fp64
    reference, including the beta * C read-modify-write epilogue."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M, N, K = 512, 768, 320
    g = torch.Generator(device="cuda").manual_seed(variant)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bt = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    dt = torch.float32 if out == "float32" else torch.bfloat16
    c0 = torch.empty(M, N, device="cuda", dtype=dt).uniform_(-1, 1, generator=g)
    c = c0.clone()
    rc = _native.lib().bk_gemm_bf16_tn_variant(
        a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N, 0.75, 0.5, 0 if out == "float32" else 2, variant,
        torch.cuda.current_stream().cuda_stream,
    )
    assert rc == 0
    torch.cuda.synchronize()
    assert_gemm_close(c, a, bt.T, out, alpha=0.75, beta=0.5, c0=c0)


def test_preload_loads_every_kernel_module(gpu):
    """bk_preload (called by the kernel broker at startup) runs one tiny
    launch per kernel module and frees what it allocated."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    before = gpu.memory_stats()["in_use"]
    assert _native.lib().bk_preload(torch.cuda.current_stream().cuda_stream) == 0
    assert gpu.memory_stats()["in_use"] == before


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("n", [1, 3, 1001, 1 << 20, 10**7 + 3])
def test_fused_rand_reduce_matches_materialised(gpu, dtype, n):
    """sum / square-sum of a lazy uniform draw (one fused Philox->reduce
    kernel) equals the reduction of the same draw once materialised."""
    g = gpu.random.default_rng(1234)
    x = g.uniform(-0.5, 2.0, n, dtype=dtype)
    fused_sq = float(gpu.sum(gpu.square(x)))
    fused_s = float(gpu.sum(x))
    host = x.numpy().astype(np.float64)  # materialises x from the same counters
    assert host.min() >= -0.5 and host.max() < 2.0
    np.testing.assert_allclose(fused_sq, (host * host).sum(), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(fused_s, host.sum(), rtol=1e-9, atol=1e-9)
    # deterministic: same seed, same bits
    g2 = gpu.random.default_rng(1234)
    assert float(gpu.sum(gpu.square(g2.uniform(-0.5, 2.0, n, dtype=dtype)))) == fused_sq


def test_lazy_draw_values_match_eager(gpu, monkeypatch):
    import importlib

    A = importlib.import_module("bee_code_interpreter_fs_amd.ops.array")  # (ops.array is also a function)
    lazy = A.Generator(77).random(4097).numpy()
    monkeypatch.setattr(A, "_LAZY_RANDOM", False)
    eager = A.Generator(77).random(4097).numpy()
    np.testing.assert_array_equal(lazy, eager)


def test_bf16_uniform_is_rounded_f32_stream(gpu):
    """Direct bf16 Philox draws == the f32 stream of the same counters,
    rounded to bf16 (what the f32-draw-then-cast path produced)."""
    import importlib

    A = importlib.import_module("bee_code_interpreter_fs_amd.ops.array")
    for n in (1, 7, 9, 4099, 1 << 20):
        direct = A.Generator(5).uniform(-1, 1, n, dtype="bfloat16").numpy()
        via_f32 = A.Generator(5).uniform(-1, 1, n, dtype="float32").astype("bfloat16").numpy()
        np.testing.assert_array_equal(direct, via_f32)


@pytest.mark.parametrize("dtype", ["float64", "float32", "bfloat16"])
@pytest.mark.parametrize("shape", [(1000, 300), (4096, 4096), (3, 70000), (70000, 3), (2, 140000), (777, 4104)])
def test_sum_mean_along_axis(gpu, dtype, shape):
    """bk.sum / bk.mean(axis=0|1) (bk_reduce_axis: column sums with chunked
    f64 partials + an ordered fold, row sums one wave per row) against fp64,
    on plain arrays and on .T views."""
    rng = np.random.default_rng(sum(shape))
    h = rng.uniform(-1, 1, shape)
    if dtype == "bfloat16":
        h = _bf16_round(h.astype(np.float32)).astype(np.float64)
    x = gpu.asarray(h, dtype)
    tol = 1e-9 if dtype == "float64" else 1e-4
    for axis in (0, 1):
        got = gpu.sum(x, axis=axis).numpy().astype(np.float64)
        np.testing.assert_allclose(got, h.sum(axis=axis), rtol=tol, atol=tol * shape[axis])
        gt = x.T.sum(axis=axis).numpy().astype(np.float64)  # transposed view: the other direction
        np.testing.assert_allclose(gt, h.T.sum(axis=axis), rtol=tol, atol=tol * shape[1 - axis])
    np.testing.assert_allclose(gpu.mean(x, axis=0).numpy().astype(np.float64), h.mean(axis=0), rtol=tol, atol=tol)
    # deterministic: same bits twice
    assert np.array_equal(gpu.sum(x, axis=0).numpy(), gpu.sum(x, axis=0).numpy())


@pytest.mark.parametrize("shape", [(256, 256, 64), (512, 768, 320), (1024, 2048, 512), (4096, 4096, 4096)])
@pytest.mark.parametrize("out", ["float32", "bfloat16"])
@pytest.mark.parametrize("pad", [0, 64])
def test_gemm_nn_kernel(gpu, shape, out, pad):
    """C = A . B with B stored [K][N] (bk_gemm_bf16_nn: the 4-wave kernel
    reading B through ds_read_b64_tr_b16 from an XOR-swizzled [k][n] LDS
    image) against fp64, beta epilogue included, ldb > N."""
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    M, N, K = shape
    ldb = N + pad
    g = torch.Generator(device="cuda").manual_seed(M + N + K + pad)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bstore = torch.empty(K, ldb, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = bstore[:, :N]
    dt = torch.float32 if out == "float32" else torch.bfloat16
    c0 = torch.empty(M, N, device="cuda", dtype=dt).uniform_(-1, 1, generator=g)
    c = c0.clone()
    lib = _native.lib()
    odt = 0 if out == "float32" else 2
    assert lib.bk_gemm_bf16_nn_ok(a.data_ptr(), bstore.data_ptr(), c.data_ptr(), M, N, K, K, ldb, N, odt) == 1
    rc = lib.bk_gemm_bf16_nn(a.data_ptr(), bstore.data_ptr(), c.data_ptr(), M, N, K, K, ldb, N, 0.75, 0.5, odt,
                             torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert_gemm_close(c, a, b, out, alpha=0.75, beta=0.5, c0=c0)


def test_gemm_nn_refuses_what_it_cannot_do(gpu):
    import torch

    from bee_code_interpreter_fs_amd.ops import _native

    lib = _native.lib()
    a = torch.zeros(300, 256, device="cuda", dtype=torch.bfloat16)
    c = torch.zeros(300, 512, device="cuda", dtype=torch.float32)
    s = torch.cuda.current_stream().cuda_stream
    # M not a tile multiple; ldb < N
    assert lib.bk_gemm_bf16_nn(a.data_ptr(), a.data_ptr(), c.data_ptr(), 300, 256, 256, 256, 256, 512, 1.0, 0.0, 0, s) == 1
    assert lib.bk_gemm_bf16_nn(a.data_ptr(), a.data_ptr(), c.data_ptr(), 256, 512, 256, 256, 256, 512, 1.0, 0.0, 0, s) == 1


@pytest.mark.parametrize("nn", ["0", "1", "auto"])
def test_matmul_row_major_b(gpu, nn, monkeypatch):
    """bk.matmul(a, b) with a plain row-major bf16 b: transpose + TN, or
    (BEE_GEMM_NN) the [K][N] kernel for tile-multiple shapes -- against fp64."""
    import numpy as np

    import sys

    arr = sys.modules["bee_code_interpreter_fs_amd.ops.array"]  # (the package exports a function named array)
    monkeypatch.setattr(arr, "_GEMM_NN", nn)
    for M, N, K in ((4096, 4096, 1024), (8192, 4096, 512), (300, 200, 136)):
        rng = np.random.default_rng(M)
        an = rng.uniform(-1, 1, (M, K)).astype(np.float32)
        bn = rng.uniform(-1, 1, (K, N)).astype(np.float32)
        a = gpu.asarray(an).astype("bfloat16")
        b = gpu.asarray(bn).astype("bfloat16")
        c = gpu.matmul(a, b, out_dtype="float32").numpy()
        ab = a.astype("float32").numpy().astype(np.float64)
        bb = b.astype("float32").numpy().astype(np.float64)
        assert gemm_error(c, ab, bb) <= 1.0, (M, N, K)


@pytest.mark.parametrize("n", [1, 2, 5, 8, 16])
@pytest.mark.parametrize("out", ["float32", "bfloat16"])
def test_gemv_shapes_take_the_skinny_kernel(gpu, n, out):
    """N <= 16 (matrix-vector products, the payload's row check): variant 8,
    A read once, against fp64 numpy."""
    from bee_code_interpreter_fs_amd.ops import _native

    m, k = 4096, 4096
    rng = np.random.default_rng(n)
    a_h = _bf16_round(rng.uniform(-1, 1, (m, k)).astype(np.float32))
    bt_h = _bf16_round(rng.uniform(-1, 1, (n, k)).astype(np.float32))
    a, bt = gpu.asarray(a_h, "bfloat16"), gpu.asarray(bt_h, "bfloat16")
    lib = _native.lib()
    assert lib.bk_gemm_bf16_pick(a.ptr, bt.ptr, a.ptr, m, n, k, k, k, n, 0 if out == "float32" else 2) == 8
    c = gpu.gemm_bf16_tn(a, bt, out_dtype=out).numpy().astype(np.float64)
    assert_gemm_close(c, a_h, bt_h.T, out)


def test_headline_gemm_check_catches_one_corrupt_tile(gpu):
    """The benchmark payload's row check (examples/benchmark_numpy_gpu.py,
    bench.gemm_row_ok) on the real kernels: a correct 4096^3 GEMM passes,
    the same C with one 256x256 tile zeroed fails."""
    import bench

    ns = {"__bk__": gpu, "__name__": "payload"}
    src = open(os.path.join(ROOT, "examples", "benchmark_numpy_gpu.py")).read()
    exec(compile(src.split("start_time = time.time()")[0].replace("import beekern as bk", "bk = __bk__"),
                 "payload", "exec"), ns)
    result, checksum, a, b, rows = ns["gpu_intensive_computation"]()
    assert bench.result_ok(float(result))
    err = float(ns["gemm_row_error"](a, b, rows))
    assert bench.gemm_row_ok(err), err
    host = gpu.matmul(a, b.T).numpy()
    assert abs(float(checksum) - float(host.astype(np.float64).sum())) < 1.0
    host[1024:1280, 2048:2304] = 0.0
    bad_rows = gpu.sum(gpu.asarray(host, "bfloat16"), axis=1)
    err_bad = float(ns["gemm_row_error"](a, b, bad_rows))
    assert not bench.gemm_row_ok(err_bad), err_bad


@pytest.mark.parametrize("dtype", ["float64", "float32", "bfloat16"])
@pytest.mark.parametrize("n", [1, 63, 4096, 1_000_003])
def test_max_abs_diff(gpu, dtype, n):
    rng = np.random.default_rng(n)
    a_h = rng.standard_normal(n)
    b_h = a_h + rng.standard_normal(n) * 1e-3
    b_h[n // 2] += 5.0  # the one outlier
    a, b = gpu.asarray(a_h, dtype), gpu.asarray(b_h, dtype)
    want = np.abs(a.numpy().astype(np.float64) - b.numpy().astype(np.float64)).max()
    assert float(gpu.max_abs_diff(a, b)) == pytest.approx(want, rel=1e-6)


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("n", [1, 4096, 1_000_003])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_max_min_propagate_nan_like_numpy(gpu, dtype, n, where):
    """One NaN anywhere (any block, the fold's first or last partial) makes
    max / min / max_abs_diff NaN, as numpy's max() does: a check of a result
    against its reference must not read a corrupt result as a small error."""
    rng = np.random.default_rng(n)
    h = rng.standard_normal(n)
    h[{"first": 0, "middle": n // 2, "last": n - 1}[where]] = np.nan
    x = gpu.asarray(h, dtype)
    y = gpu.asarray(np.zeros(n), dtype)
    assert np.isnan(np.abs(h).max())  # numpy's answer
    assert np.isnan(float(gpu.amax(x))) and np.isnan(float(gpu.amin(x)))
    assert np.isnan(float(gpu.max_abs_diff(x, y))) and np.isnan(float(gpu.max_abs_diff(y, x)))
    # elementwise maximum / minimum: NaN in either operand
    m = gpu.maximum(y, x).numpy()
    assert np.array_equal(np.isnan(m), np.isnan(np.maximum(np.zeros(n), h)))
    m = gpu.minimum(x, y).numpy()
    assert np.array_equal(np.isnan(m), np.isnan(np.minimum(h, np.zeros(n))))


SEGMENT_PROBE = r"""
import ctypes, random
import numpy as np
from bee_code_interpreter_fs_amd import ops
from bee_code_interpreter_fs_amd.ops import _native
ops.init(0)
lib = _native.lib()
lib.bk_reserve.argtypes = [ctypes.c_int64]
assert lib.bk_reserve(1 << 30) == 0
rng = random.Random(5)
live = {}
for step in range(400):
    if live and (rng.random() < 0.45 or len(live) > 40):
        k = rng.choice(list(live))
        arr, val = live.pop(k)
        assert float(ops.amax(arr)) == val and float(ops.amin(arr)) == val, (step, k)  # nobody wrote over it
        del arr
    else:
        n = rng.choice([1 << 18, 3 << 19, 1 << 20, 5 << 20, 1 << 23, 3 << 24]) // 8  # bytes -> f64 elements
        val = float(step)
        live[step] = (ops.full((n,), val, "float64"), val)
for k, (arr, val) in live.items():
    assert float(ops.amax(arr)) == val and float(ops.amin(arr)) == val
live.clear()
ops.synchronize()
st = (ctypes.c_int64 * 4)()
lib.bk_memory_stats(st)
# everything back and coalesced: one 1 GiB block fits again without a new segment
big = ops.empty(((1 << 30) - (2 << 20)) // 8, "float64")
lib.bk_memory_stats(st)
print("ok", st[0], st[1])
"""


def test_broker_segment_allocator_reuses_and_coalesces(gpu):
    """bk_reserve switches large blocks to best-fit segments (what the kernel
    broker runs on): random alloc / free churn over 256 KiB..48 MiB blocks
    never hands out overlapping memory, and once everything is freed the
    segment coalesces back into one extent (a ~1 GiB block fits in it)."""
    import subprocess
    import sys

    p = subprocess.run([sys.executable, "-c", SEGMENT_PROBE], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0 and p.stdout.startswith("ok"), p.stdout + p.stderr[-3000:]
