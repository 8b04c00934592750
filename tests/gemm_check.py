"""The error bound a bf16-operand GEMM must meet.

Products of bf16 operands are exact in f32 (8 + 8 significant bits), so an
f32-output GEMM differs from the fp64 product of the same (rounded)
operands only by its f32 accumulation: elementwise well below
``1e-5 * (|A| @ |B|)``.  A bf16 output is that f32 result rounded to
nearest, ``<= 2**-8`` of its magnitude on top.  The beta epilogue
``alpha * A @ B + beta * C0`` adds one f32 rounding of a value bounded by
``|alpha| |A| @ |B| + |beta| |C0|``.  The old tolerances (``rtol=1e-2`` plus
``2e-3 * sqrt(K)`` absolute) were ~1000x looser; a product missing one
64-deep K tile fails this bound (tests/test_kernels_gpu.py
test_gemm_bound_catches_a_missing_k_tile)."""

import numpy as np

F32_REL = 1e-5
BF16_REL = 2.0 ** -8


def _np(x):
    if hasattr(x, "detach"):  # a torch tensor
        return x.detach().double().cpu().numpy()
    return np.asarray(x, dtype=np.float64)


def gemm_error(c, a, b, out="float32", alpha=1.0, beta=0.0, c0=None):
    """max over elements of |C - ref| / bound; <= 1 passes.  ``a`` is M x K,
    ``b`` K x N (the fp64 values of the bf16 operands)."""
    c, a, b = _np(c), _np(a), _np(b)
    ref = alpha * (a @ b)
    mag = abs(alpha) * (np.abs(a) @ np.abs(b))
    if c0 is not None and beta != 0.0:
        c0 = _np(c0)
        ref = ref + beta * c0
        mag = mag + abs(beta) * np.abs(c0)
    bound = F32_REL * mag
    if out != "float32":
        bound = BF16_REL * np.abs(ref) + 1.01 * bound
    err = np.abs(c - ref)
    return float(np.max(err / np.maximum(bound, 1e-300))) if err.size else 0.0


def assert_gemm_close(c, a, b, out="float32", alpha=1.0, beta=0.0, c0=None):
    r = gemm_error(c, a, b, out, alpha, beta, c0)
    assert r <= 1.0, f"GEMM error {r:.3g}x its bound (out={out})"
