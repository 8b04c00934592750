"""beekern — hand-written CDNA4 (gfx950) kernels behind a numpy-like API.

Exposed to sandboxed code as the top-level module ``beekern`` (see
``runtime/sandbox_modules/beekern.py``).  Kernels: Philox RNG, elementwise
(square & friends), deterministic reductions (sum, fused square-sum, dot,
min/max), bf16 MFMA GEMM and f64 / f32 MFMA GEMM at numpy's precision — source in ``csrc/kernels``.
"""

from ._native import BeekernError, QuotaExceeded, library_path  # noqa: F401
from .array import (  # noqa: F401
    DeviceArray,
    Generator,
    Timer,
    abs,
    add,
    amax,
    amin,
    array,
    asarray,
    cos,
    device_info,
    divide,
    dot,
    driver_name,
    empty,
    empty_cache,
    exp,
    from_numpy,
    from_torch,
    full,
    gemm_bf16_tn,
    init,
    is_initialized,
    log,
    matmul,
    matmul_fp,
    max_abs_diff,
    maximum,
    mean,
    memory_stats,
    minimum,
    multiply,
    negative,
    normalize_dtype,
    ones,
    power,
    random,
    relu,
    set_lazy_random,
    set_quota,
    sigmoid,
    sin,
    sqrt,
    square,
    square_sum,
    subtract,
    sum,
    synchronize,
    tanh,
    to_torch,
    zeros,
)

float32 = "float32"
float64 = "float64"
bfloat16 = "bfloat16"
