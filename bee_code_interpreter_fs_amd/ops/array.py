"""``DeviceArray``: a minimal numpy-like array in MI355X HBM, driven by the
hand-written beekern kernels.

Sandboxed user code calls these in place of numpy (BASELINE.json north
star).  The benchmark payload `examples/benchmark-numpy.py:18-22` becomes::

    import beekern as bk
    x = bk.random.rand(10**8)          # Philox kernel, f64, stays in HBM
    result = bk.sum(bk.square(x))      # fused square+sum: one HBM read pass

``square`` (and ``x * x`` / ``x ** 2``) returns a *lazy* array: if the only
consumer is a reduction the square is fused into it (no 800 MB temporary);
any other use materialises it with the elementwise kernel.

Kernels run through a driver (``ops/driver.py``): in-process HIP (native) or
the executor's kernel broker (light sandboxes, no HIP context of their own).
"""

from __future__ import annotations

import math
import os
import struct
import threading
from typing import Any, Optional, Sequence, Tuple

from ._lazy import is_integer, is_number, np, scalar
from ._native import DTYPE_CODES, DTYPE_SIZES, BeekernError, QuotaExceeded  # noqa: F401
from .driver import make_driver

Shape = Tuple[int, ...]

_UNARY = {
    "square": 0, "abs": 1, "negative": 2, "sqrt": 3, "exp": 4, "log": 5, "relu": 6,
    "sin": 7, "cos": 8, "tanh": 9, "sigmoid": 10, "copy": 11,
}
_BINARY = {"add": 0, "subtract": 1, "multiply": 2, "divide": 3, "maximum": 4, "minimum": 5, "power": 6}
_REDUCE = {"sum": 0, "square_sum": 1, "abs_sum": 2, "max": 3, "min": 4, "dot": 5, "max_abs_diff": 6}
_SUPPORTED = ("float32", "float64", "bfloat16")

_state_lock = threading.Lock()
_driver = None


def normalize_dtype(dtype: Any) -> str:
    if dtype is None:
        return "float64"
    if isinstance(dtype, str):
        name = {"bf16": "bfloat16", "f32": "float32", "f64": "float64", "double": "float64", "float": "float64"}.get(
            dtype, dtype
        )
    else:
        name = str(getattr(dtype, "name", None) or np.dtype(dtype).name)
        name = name.replace("torch.", "")
    if name not in _SUPPORTED:
        raise TypeError(f"unsupported dtype {dtype!r}; beekern supports {_SUPPORTED}")
    return name


def init(device: Optional[int] = None, lazy: bool = False) -> int:
    """Initialise the driver (HIP context on ``device``, or a broker session);
    idempotent.  Sandboxes do this while waiting in the warm pool.  ``lazy``
    (broker driver only) defers opening the session to the first request."""
    global _driver
    if _driver is not None:
        return _driver.device
    with _state_lock:
        if _driver is None:
            d = make_driver()
            dev = int(os.environ.get("BEE_DEVICE", "0")) if device is None else int(device)
            if lazy and d.name == "broker":
                d.init(dev, lazy=True)
            else:
                d.init(dev)
            _driver = d
    return _driver.device


def driver():
    if _driver is None:
        init()
    return _driver


def driver_name() -> str:
    return driver().name


def is_initialized() -> bool:
    return _driver is not None


def synchronize() -> None:
    if _driver is not None:
        _driver.sync()


def memory_stats() -> dict:
    return driver().memory_stats()


def set_quota(nbytes: int) -> None:
    driver().set_quota(int(nbytes))


def empty_cache() -> None:
    driver().empty_cache()


def device_info() -> dict:
    return driver().device_info()


class _Buffer:
    """Owns one device allocation (pointer or broker handle)."""

    __slots__ = ("ptr", "nbytes", "_owner", "_drv", "__weakref__")

    def __init__(self, nbytes: int, ptr: Optional[int] = None, owner: Any = None) -> None:
        self.nbytes = int(nbytes)
        self._owner = owner
        self._drv = driver()
        self.ptr = int(ptr) if ptr is not None else self._drv.malloc(max(self.nbytes, 1))

    def __del__(self) -> None:
        if self._owner is None and getattr(self, "ptr", 0):
            try:
                self._drv.free(self.ptr)
            except Exception:
                pass


class DeviceArray:
    """Contiguous row-major array in device memory (or a lazy unary view)."""

    __array_priority__ = 1000

    def __init__(self, shape: Sequence[int], dtype: str, buffer: Optional[_Buffer] = None, lazy=None, strides_t=False):
        self.shape: Shape = tuple(int(s) for s in shape)
        self.dtype = normalize_dtype(dtype)
        # until materialised: ("square", src), or ("rand", kind, seed, offset,
        # lo, hi) -- a draw whose values are fixed by its counter range
        self._lazy = lazy
        self._transposed = strides_t  # 2-D transposed view of a contiguous buffer
        if buffer is None and lazy is None:
            buffer = _Buffer(self.nbytes)
        self._buf = buffer

    @property
    def size(self) -> int:
        return int(math.prod(self.shape)) if self.shape else 1

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def itemsize(self) -> int:
        return DTYPE_SIZES[self.dtype]

    @property
    def nbytes(self) -> int:
        return self.size * self.itemsize

    @property
    def ptr(self) -> int:
        self._materialize()
        return self._buf.ptr  # type: ignore[union-attr]

    @property
    def code(self) -> int:
        return DTYPE_CODES[self.dtype]

    def __len__(self) -> int:
        if not self.shape:
            raise TypeError("len() of a 0-d array")
        return self.shape[0]

    def __repr__(self) -> str:
        kind = "lazy " if self._lazy else ""
        return f"DeviceArray({kind}shape={self.shape}, dtype={self.dtype})"

    def _materialize(self) -> "DeviceArray":
        if self._lazy is not None:
            if self._lazy[0] == "rand":
                _, kind, seed, off, lo, hi = self._lazy
                self._buf = _Buffer(self.nbytes)
                driver().rand(kind, self._buf.ptr, self.size, self.code, seed, off, lo, hi)
            else:
                op, src = self._lazy
                self._buf = _Buffer(self.nbytes)
                driver().unary(_UNARY[op], self.code, src.ptr, self._buf.ptr, self.size)
            self._lazy = None
        if self._transposed:
            rows, cols = self.shape[1], self.shape[0]  # underlying buffer is (rows, cols)
            src = self._buf
            out = _Buffer(self.nbytes)  # on-device transpose, 2/4/8-byte elements
            driver().transpose(src.ptr, out.ptr, rows, cols, cols, rows, self.code, self.code)
            self._buf = out
            self._transposed = False
        return self

    def numpy(self) -> np.ndarray:
        self._materialize()
        return _download(self._buf, self.shape, self.dtype)

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    # numpy functions and ufuncs on a device array run on the kernels where
    # one computes what numpy would; the rest copy to the host once, with a
    # warning (ops/npinterop.py) -- not silently through __array__
    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        from .npinterop import array_ufunc

        return array_ufunc(_binding(), ufunc, method, inputs, kwargs)

    def __array_function__(self, func, types, args, kwargs):
        from .npinterop import array_function

        return array_function(_binding(), func, types, args, kwargs)

    def tolist(self):
        return self.numpy().tolist()

    def item(self):
        if self.size != 1:
            raise ValueError("item() needs a size-1 array")
        return self.numpy().reshape(()).item()

    def __float__(self) -> float:
        return float(self.item())

    def reshape(self, *shape) -> "DeviceArray":
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        shape = list(shape)
        if -1 in shape:
            known = math.prod(s for s in shape if s != -1)
            shape[shape.index(-1)] = self.size // max(known, 1)
        if math.prod(shape) != self.size:
            raise ValueError(f"cannot reshape {self.shape} to {tuple(shape)}")
        self._materialize()
        return DeviceArray(shape, self.dtype, buffer=self._buf)

    @property
    def T(self) -> "DeviceArray":
        if self.ndim != 2:
            raise ValueError("T needs a 2-D array")
        self._materialize()
        return DeviceArray((self.shape[1], self.shape[0]), self.dtype, buffer=self._buf, strides_t=True)

    def astype(self, dtype) -> "DeviceArray":
        dt = normalize_dtype(dtype)
        if dt == self.dtype:
            return self.copy()
        self._materialize()
        out = DeviceArray(self.shape, dt)
        driver().cast(self.code, out.code, self.ptr, out.ptr, self.size)
        return out

    def copy(self) -> "DeviceArray":
        return _unary("copy", self)

    def sum(self, axis: Optional[int] = None):
        return sum(self, axis)

    def mean(self, axis: Optional[int] = None):
        return mean(self, axis)

    def max(self):
        return _reduce("max", self)

    def min(self):
        return _reduce("min", self)

    def __add__(self, o): return _binary("add", self, o)
    def __radd__(self, o): return _binary("add", self, o)
    def __sub__(self, o): return _binary("subtract", self, o)
    def __rsub__(self, o): return _binary("subtract", self, o, reversed_=True)
    def __mul__(self, o):
        if o is self:
            return square(self)
        return _binary("multiply", self, o)
    def __rmul__(self, o): return _binary("multiply", self, o)
    def __truediv__(self, o): return _binary("divide", self, o)
    def __rtruediv__(self, o): return _binary("divide", self, o, reversed_=True)
    def __pow__(self, o):
        if isinstance(o, (int, float)) and o == 2:
            return square(self)
        return _binary("power", self, o)
    def __neg__(self): return _unary("negative", self)
    def __abs__(self): return _unary("abs", self)
    def __matmul__(self, o): return matmul(self, o)


_BINDING = []


def _binding():
    """DeviceArray's plug into the numpy protocols (ops/npinterop.py)."""
    if not _BINDING:
        from .npinterop import Binding

        def mine(x):
            return isinstance(x, DeviceArray)

        _BINDING.append(Binding(dev=lambda x: x if mine(x) else None, box=lambda d: d,
                                host=lambda x: x.numpy(), is_mine=mine))
    return _BINDING[0]


def _np_dtype(dtype: str):
    return {"float32": np.float32, "float64": np.float64}[dtype]


def _np_view_dtype(dtype: str):
    return np.uint16 if dtype == "bfloat16" else _np_dtype(dtype)


def _download(buf: _Buffer, shape: Shape, dtype: str) -> np.ndarray:
    host = np.empty(shape, dtype=_np_view_dtype(dtype))
    driver().d2h(buf.ptr, host)
    if dtype == "bfloat16":
        return (host.astype(np.uint32) << 16).view(np.float32)
    return host


def _upload(host: np.ndarray, dtype: str) -> _Buffer:
    host = np.ascontiguousarray(host)
    buf = _Buffer(host.nbytes)
    driver().h2d(buf.ptr, host)
    return buf


def _f32_bits_to_bf16(u: int) -> int:
    """One f32 bit pattern -> bf16 bits, round to nearest even (NaN -> 0x7FC0),
    as _f32_to_bf16_bits does element-wise."""
    if (u & 0x7F800000) == 0x7F800000 and (u & 0x007FFFFF):
        return 0x7FC0
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF


def _f32_to_bf16_bits(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    rounded = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    out = rounded.astype(np.uint16)
    nan = np.isnan(a)
    if nan.any():
        out[nan] = 0x7FC0
    return out


# ---- constructors -------------------------------------------------------------------

def empty(shape, dtype="float64") -> DeviceArray:
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    return DeviceArray(shape, dtype)


def full(shape, value: float, dtype="float64") -> DeviceArray:
    a = empty(shape, dtype)
    # the fill's bit pattern (no numpy: see ops/_lazy.py)
    if a.dtype == "float64":
        pattern, width = struct.unpack("<Q", struct.pack("<d", float(value)))[0], 8
    elif a.dtype == "float32":
        pattern, width = struct.unpack("<I", struct.pack("<f", float(value)))[0], 4
    else:
        pattern, width = _f32_bits_to_bf16(struct.unpack("<I", struct.pack("<f", float(value)))[0]), 2
    driver().fill(a.ptr, a.nbytes, pattern, width)
    return a


def zeros(shape, dtype="float64") -> DeviceArray:
    return full(shape, 0.0, dtype)


def ones(shape, dtype="float64") -> DeviceArray:
    return full(shape, 1.0, dtype)


def asarray(obj, dtype=None) -> DeviceArray:
    if isinstance(obj, DeviceArray):
        return obj if dtype is None or normalize_dtype(dtype) == obj.dtype else obj.astype(dtype)
    if _is_torch_tensor(obj):
        return from_torch(obj) if dtype is None else from_torch(obj).astype(dtype)
    host = np.asarray(obj)
    dt = normalize_dtype(dtype if dtype is not None else (host.dtype if host.dtype.kind == "f" else "float64"))
    if dt == "bfloat16":
        buf = _upload(_f32_to_bf16_bits(host.astype(np.float32)), "bfloat16")
    else:
        buf = _upload(host.astype(_np_dtype(dt), copy=False), dt)
    return DeviceArray(host.shape, dt, buffer=buf)


from_numpy = asarray
array = asarray


def _is_torch_tensor(x) -> bool:
    t = type(x)
    return t.__module__.startswith("torch") and t.__name__ in ("Tensor", "Parameter")


def from_torch(t) -> DeviceArray:
    """Zero-copy view of a contiguous HIP torch tensor when this process owns
    the HIP context; a host copy in broker mode."""
    dt = normalize_dtype(str(t.dtype).replace("torch.", ""))
    if t.is_cuda and driver().name == "native":
        t = t.contiguous()
        return DeviceArray(tuple(t.shape), dt, buffer=_Buffer(t.numel() * t.element_size(), ptr=t.data_ptr(), owner=t))
    host = t.detach().cpu()
    if dt == "bfloat16":
        import torch

        return asarray(host.to(torch.float32).numpy(), "bfloat16")
    return asarray(host.numpy(), dt)


def to_torch(a: DeviceArray):
    import torch

    host = a.numpy()
    dt = {"float32": torch.float32, "float64": torch.float64, "bfloat16": torch.bfloat16}[a.dtype]
    return torch.from_numpy(host).to(device="cuda", dtype=dt)


# ---- elementwise / reductions ------------------------------------------------------

def _as_operand(x) -> DeviceArray:
    return x if isinstance(x, DeviceArray) else asarray(x)


def _unary(op: str, x) -> DeviceArray:
    x = _as_operand(x)._materialize()
    out = DeviceArray(x.shape, x.dtype)
    driver().unary(_UNARY[op], x.code, x.ptr, out.ptr, x.size)
    return out


def square(x) -> DeviceArray:
    """Lazy x**2: fused into a following reduction, else materialised.  A
    still-lazy uniform draw stays lazy underneath (sum(square(rand)) is one
    fused Philox->square->reduce kernel)."""
    x = _as_operand(x)
    if not _lazy_uniform(x):
        x = x._materialize()
    return DeviceArray(x.shape, x.dtype, lazy=("square", x))


def _binary(op: str, a, b, reversed_: bool = False) -> DeviceArray:
    a = _as_operand(a)._materialize()
    if is_number(b):
        out = DeviceArray(a.shape, a.dtype)
        driver().binary(_BINARY[op], a.code, 2 if reversed_ else 1, a.ptr, 0, float(b), out.ptr, a.size)
        return out
    b = _as_operand(b)._materialize()
    if b.shape != a.shape or b.dtype != a.dtype:
        if b.size == 1:
            return _binary(op, a, float(b.item()), reversed_)
        raise ValueError(f"beekern {op}: shapes/dtypes must match ({a.shape} {a.dtype} vs {b.shape} {b.dtype})")
    if reversed_:
        a, b = b, a
    out = DeviceArray(a.shape, a.dtype)
    driver().binary(_BINARY[op], a.code, 0, a.ptr, b.ptr, 0.0, out.ptr, a.size)
    return out


def _reduce(op: str, x: DeviceArray, y: Optional[DeviceArray] = None) -> np.float64:
    return scalar(driver().reduce(_REDUCE[op], x.code, x.ptr, y.ptr if y is not None else 0, x.size))


def _lazy_uniform(x: DeviceArray) -> bool:
    # fused reductions exist for the f64 / f32 streams (bf16 draws materialise)
    return x._lazy is not None and x._lazy[0] == "rand" and x._lazy[1] == 0 and x.dtype != "bfloat16"


def _rand_reduce(op: str, x: DeviceArray) -> np.float64:
    """Reduce a still-lazy uniform draw in one fused Philox->reduce kernel
    (bk_rand_reduce): the values are the ones materialising x would store."""
    _, _, seed, off, lo, hi = x._lazy
    return scalar(driver().rand_reduce(_REDUCE[op], x.code, x.size, seed, off, lo, hi))


def _reduce_axis(op: str, x: DeviceArray, axis: int):
    """sum / mean of a 2-D array along ``axis`` (numpy semantics: axis 0
    collapses the rows -> one value per column).  f64 in -> f64 out; f32 and
    bf16 in -> f32 out; f64 accumulation (bk_reduce_axis)."""
    if x.ndim == 1:
        if axis not in (0, -1):
            raise ValueError(f"axis {axis} is out of bounds for a 1-D array")
        return sum(x) if op == "sum" else mean(x)  # numpy: a scalar
    if x.ndim != 2:
        raise ValueError("axis reductions support 1-D and 2-D arrays")
    axis = axis + 2 if axis < 0 else axis
    if axis not in (0, 1):
        raise ValueError(f"axis {axis} is out of bounds for a 2-D array")
    if x._lazy is not None:
        x._materialize()
    rows, cols = x.shape
    if x._transposed:  # a .T view: the buffer is (cols, rows) -- reduce the other way
        rows, cols, axis = cols, rows, 1 - axis
    out = DeviceArray((cols if axis == 0 else rows,), "float64" if x.dtype == "float64" else "float32")
    driver().reduce_axis(0 if op == "sum" else 1, x.code, x._buf.ptr, out.ptr, rows, cols, cols, axis)  # type: ignore[union-attr]
    return out


def sum(x, axis: Optional[int] = None):  # noqa: A001 - numpy-compatible name
    x = _as_operand(x)
    if axis is not None:
        return _reduce_axis("sum", x, int(axis))
    if x._lazy is not None and x._lazy[0] == "square":
        base = x._lazy[1]
        if _lazy_uniform(base):
            return _rand_reduce("square_sum", base)  # neither the draw nor x**2 materialised
        return _reduce("square_sum", base)  # fused: x**2 never materialised
    if _lazy_uniform(x):
        return _rand_reduce("sum", x)
    return _reduce("sum", x._materialize())


def square_sum(x) -> np.float64:
    x = _as_operand(x)
    if _lazy_uniform(x):
        return _rand_reduce("square_sum", x)
    return _reduce("square_sum", x._materialize())


def mean(x, axis: Optional[int] = None):
    x = _as_operand(x)
    if axis is not None:
        return _reduce_axis("mean", x, int(axis))
    return sum(x) / x.size


def dot(a, b):
    a, b = _as_operand(a), _as_operand(b)
    if a.ndim == 2 or b.ndim == 2:
        return matmul(a, b)  # (.T views stay views: the GEMMs read them in place)
    a, b = a._materialize(), b._materialize()
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("dot: 1-D operands must match in shape and dtype")
    return _reduce("dot", a, b)


def max_abs_diff(a, b) -> np.float64:
    """max(|a - b|) in one pass (no a - b array): e.g. a result against its
    reference.  Same shape and dtype."""
    a, b = _as_operand(a)._materialize(), _as_operand(b)._materialize()
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("max_abs_diff: operands must match in shape and dtype")
    return _reduce("max_abs_diff", a, b)


def amax(x): return _reduce("max", _as_operand(x)._materialize())
def amin(x): return _reduce("min", _as_operand(x)._materialize())


def _make_unary(name):
    def fn(x):
        return _unary(name, x)

    fn.__name__ = name
    return fn


abs = _make_unary("abs")  # noqa: A001
negative = _make_unary("negative")
sqrt = _make_unary("sqrt")
exp = _make_unary("exp")
log = _make_unary("log")
relu = _make_unary("relu")
sin = _make_unary("sin")
cos = _make_unary("cos")
tanh = _make_unary("tanh")
sigmoid = _make_unary("sigmoid")


def add(a, b): return _binary("add", a, b)
def subtract(a, b): return _binary("subtract", a, b)
def multiply(a, b): return _binary("multiply", a, b)
def divide(a, b): return _binary("divide", a, b)
def maximum(a, b): return _binary("maximum", a, b)
def minimum(a, b): return _binary("minimum", a, b)
def power(a, b): return _binary("power", a, b)


# ---- matmul --------------------------------------------------------------------------

# The [K][N] kernel (bk_gemm_bf16_nn) reads B in place; the alternative is a
# transpose pass (4*K*N bytes of HBM traffic) then the TN kernel, which runs
# 7-10% faster than the [K][N] one.  The pass costs ~600/M of the GEMM, so
# reading in place wins below M ~ 6k.  Measured on MI355X, TFLOP/s, [K][N]
# kernel vs transpose + TN (hipBLASLt's NN in brackets,
# profiles/archive/r2_s3_gemm_nn_sweep.log):
#   M=N=4096,  K=512..4096: 715/949/1132/1229/1298 vs 574/771/1029/1154/1218
#                           (659/935/1140/1256/1302)
#   2048x8192x2048: 1211 vs 1014 (1195)
#   M=N=8192,  K=1024..8192: 1081/1242/1286/1298 vs 1091/1252/1328/1325
#   16384x4096x1024: 1104 vs 1108
# BEE_GEMM_NN: auto (M below _NN_MAX_M), 1 (whenever the shape allows), 0 (never)
_GEMM_NN = os.environ.get("BEE_GEMM_NN", "auto")
_NN_MAX_M = 6144


def _use_nn(M: int) -> bool:
    return _GEMM_NN == "1" or (_GEMM_NN == "auto" and M < _NN_MAX_M)


def _fp_dtype(x) -> bool:
    return x.dtype in ("float32", "float64")


# f32 products take the six-piece bf16 split (csrc/kernels/gemm_fp.hip
# bk_gemm_f32x6: f32-level error at the bf16 MFMA's rate) above 2^33
# multiply-adds with M, N >= 256; smaller ones, and any product whose
# workspace the HBM quota refuses, run on the f32 MFMA.  Measured medians,
# split vs f32 kernel (profiles/r6_gemm_fp_sweep.jsonl, f32 kernel with the
# buffer loads): 1024^3 81 vs 26 us, 1536^3 113 vs 80, 2048^3 (= 2^33) 153
# vs 138, 4000x3000x1000 153 vs 191, 3072^3 426 vs 424 (level), 4096^3 696
# vs 1005.  BEE_GEMM_F32X6: auto | 1 (whenever the shape allows) | 0 (never).
_F32X6 = os.environ.get("BEE_GEMM_F32X6", "auto")
_F32X6_MIN_MACS = (1 << 33) + 1


def f32x6_workspace_bytes(M: int, N: int, K: int) -> int:
    """Workspace of the split product: a 256-byte header, then A' [M][6 Kp]
    and B' [N][6 Kp] in bf16, Kp = K rounded up to 64 (broker_core.hpp)."""
    return 256 + 12 * ((K + 63) // 64 * 64) * (M + N)


def _use_f32x6(M: int, N: int, K: int) -> bool:
    if _F32X6 == "0" or 6 * ((K + 63) // 64 * 64) > (1 << 22):
        return False
    return _F32X6 == "1" or (min(M, N) >= 256 and M * N * K >= _F32X6_MIN_MACS)


def matmul_fp(a, b) -> DeviceArray:
    """C = A @ B in numpy's precision: f64 operands on the f64 MFMA
    (``v_mfma_f64_16x16x4_f64``), f32 on the exact f32 MFMA
    (``v_mfma_f32_16x16x4_f32``) or, for large products, on the bf16 MFMA
    through the six-piece split (f32-level error, :func:`f32x6_workspace_bytes`),
    mixed f32/f64 promoted to f64 as numpy does (``csrc/kernels/gemm_fp.hip``).  numpy's 1-D rules: a 1-D ``a`` is
    a row vector, a 1-D ``b`` a column, and that axis is dropped from the
    result.  ``.T`` views are read in place (no transpose pass)."""
    a = _as_operand(a)
    b = _as_operand(b)
    if not (_fp_dtype(a) and _fp_dtype(b)) or a.ndim not in (1, 2) or b.ndim not in (1, 2):
        raise ValueError(f"matmul_fp: f32/f64 operands of 1 or 2 dimensions, got {a.shape} {a.dtype} @ {b.shape} {b.dtype}")
    dt = "float64" if "float64" in (a.dtype, b.dtype) else "float32"
    a1, b1 = a.ndim == 1, b.ndim == 1
    if a1:
        a = a.reshape(1, a.shape[0])
    if b1:
        b = b.reshape(b.shape[0], 1)
    if a.shape[1] != b.shape[0]:
        raise ValueError(f"matmul: incompatible shapes {a.shape} @ {b.shape}")
    if a.dtype != dt:
        a = a.astype(dt)
    if b.dtype != dt:
        b = b.astype(dt)
    M, K = a.shape
    N = b.shape[1]
    out_shape = tuple(s for s, drop in ((M, a1), (N, b1)) if not drop)
    if M == 0 or N == 0 or K == 0:
        return zeros(out_shape, dt)  # (numpy: an empty product, or zeros for K == 0)
    # a .T view is never lazy (T materialises first): its buffer is the
    # row-major transpose, read as is with the transposed-operand flag
    ta, tb = a._transposed, b._transposed
    a_ptr = a._buf.ptr if ta else a.ptr  # type: ignore[union-attr]
    b_ptr = b._buf.ptr if tb else b.ptr  # type: ignore[union-attr]
    c = DeviceArray((M, N), dt)
    lda, ldb = (M if ta else K), (K if tb else N)
    ws = None
    if dt == "float32" and _use_f32x6(M, N, K):
        nbytes = f32x6_workspace_bytes(M, N, K)
        try:
            ws = DeviceArray((nbytes // 2,), "bfloat16")
        except QuotaExceeded:
            ws = None  # (no room for the split operands: the f32 MFMA needs none)
    if ws is not None:
        driver().gemm_f32x6(ta, tb, a_ptr, b_ptr, c.ptr, M, N, K, lda, ldb, N, ws.ptr, nbytes)
        del ws  # (freed in stream order)
    else:
        driver().gemm_fp(DTYPE_CODES[dt], ta, tb, a_ptr, b_ptr, c.ptr, M, N, K, lda, ldb, N)
    return c.reshape(out_shape) if out_shape != (M, N) else c


def matmul(a, b, out_dtype: Optional[str] = None) -> DeviceArray:
    """C = A @ B.

    f32 / f64 operands (and no ``out_dtype``): numpy's precision on the
    full-precision MFMA GEMM (:func:`matmul_fp`).  A bf16 operand or an
    explicit ``out_dtype``: the bf16 MFMA GEMM (f32 accumulate; f32 / f64
    operands are rounded to bf16), bf16 result by default.

    On the bf16 path ``b.T`` views of a row-major [N, K] buffer are used as
    is (the TN kernels); a plain row-major bf16 ``b`` is read in place by the
    [K][N] kernel for tile-multiple shapes with M below ~6k (BEE_GEMM_NN),
    else transposed once on device (15 us at 4096^2) for the TN kernel; an
    f32/f64 ``b`` is converted and transposed in the same pass.
    """
    a = _as_operand(a)
    b = _as_operand(b)
    if out_dtype is None:
        if _fp_dtype(a) and _fp_dtype(b):
            return matmul_fp(a, b)
        out_dtype = "bfloat16"
    if a.ndim != 2 or b.ndim != 2 or a.shape[1] != b.shape[0]:
        raise ValueError(f"matmul: incompatible shapes {a.shape} @ {b.shape}")
    M, K = a.shape
    N = b.shape[1]
    if a.dtype != "bfloat16":
        a = a.astype("bfloat16")
    a._materialize()
    if b._transposed and b.dtype == "bfloat16" and b._lazy is None:
        bt_ptr = b._buf.ptr  # the underlying buffer already is Bt[N, K]
        keep = b
    elif b._transposed and b.dtype in ("float32", "float64") and b._lazy is None:
        # the underlying buffer is Bt[N, K] already: only the conversion
        keep = DeviceArray((N, K), "bfloat16")
        driver().cast(b.code, DTYPE_CODES["bfloat16"], b._buf.ptr, keep.ptr, N * K)
        bt_ptr = keep.ptr
    elif b.dtype in ("float32", "float64") and not b._transposed and K % 8 == 0 and N % 8 == 0 and \
            (driver().name == "broker" or b.ptr % 16 == 0):
        # one pass: f32/f64 B[K, N] -> bf16 Bt[N, K] (broker handles are allocation bases: 16-B aligned)
        keep = DeviceArray((N, K), "bfloat16")
        driver().transpose(b.ptr, keep.ptr, K, N, N, K, DTYPE_CODES[b.dtype])
        bt_ptr = keep.ptr
    else:
        if b.dtype != "bfloat16":
            b = b.astype("bfloat16")
        b._materialize()
        out_dtype = normalize_dtype(out_dtype)
        from .driver import nn_shape_ok

        d = driver()
        if _use_nn(M) and hasattr(d, "gemm_nn") and nn_shape_ok(M, N, K, K, N, N, out_dtype == "bfloat16") and \
                (d.name == "broker" or (a.ptr % 16 == 0 and b.ptr % 16 == 0)):
            # B[K, N] read in place through transposed LDS reads: no transpose pass
            c = DeviceArray((M, N), out_dtype)
            d.gemm_nn(a.ptr, b.ptr, c.ptr, M, N, K, K, N, N, 1.0, 0.0, DTYPE_CODES[out_dtype])
            return c
        keep = DeviceArray((N, K), "bfloat16")
        driver().transpose(b.ptr, keep.ptr, K, N, N, K)
        bt_ptr = keep.ptr
    out_dtype = normalize_dtype(out_dtype)
    c = DeviceArray((M, N), out_dtype)
    driver().gemm(a.ptr, bt_ptr, c.ptr, M, N, K, K, K, N, 1.0, 0.0, DTYPE_CODES[out_dtype])
    del keep
    return c


def gemm_bf16_tn(a: DeviceArray, bt: DeviceArray, out_dtype: str = "bfloat16", alpha: float = 1.0) -> DeviceArray:
    """Raw C = alpha * A . Bt^T with both operands already bf16 [M,K] / [N,K]."""
    M, K = a.shape
    N = bt.shape[0]
    out_dtype = normalize_dtype(out_dtype)
    c = DeviceArray((M, N), out_dtype)
    driver().gemm(a.ptr, bt.ptr, c.ptr, M, N, K, K, K, N, float(alpha), 0.0, DTYPE_CODES[out_dtype])
    return c


# ---- random ----------------------------------------------------------------------------

_LAZY_RANDOM = os.environ.get("BEE_LAZY_RANDOM", "1") != "0"


def set_lazy_random(enabled: bool) -> bool:
    """Uniform draws are lazy by default: generated on first use, and fused
    into a reduction that consumes them directly.  ``False`` materialises
    every draw in HBM at once (numpy's data movement: the reference
    payload's 800 MB array).  Returns the previous setting."""
    global _LAZY_RANDOM
    prev, _LAZY_RANDOM = _LAZY_RANDOM, bool(enabled)
    return prev


class Generator:
    """Counter-based Philox4x32-10 stream on the device (numpy.random subset)."""

    def __init__(self, seed: Optional[int] = None) -> None:
        self.seed(seed)

    def seed(self, seed: Optional[int] = None) -> None:
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self._seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self._offset = 0

    def _advance(self, n: int, per_call: int) -> int:
        off = self._offset
        self._offset += (n + per_call - 1) // per_call
        return off

    def random(self, size=None, dtype="float64") -> DeviceArray:
        return self.uniform(0.0, 1.0, size, dtype)

    def rand(self, *shape, dtype="float64") -> DeviceArray:
        return self.uniform(0.0, 1.0, shape or (1,), dtype)

    def _draw(self, kind: int, a: float, b: float, size, dtype) -> DeviceArray:
        shape = _shape_of(size)
        dt = normalize_dtype(dtype)
        if dt == "bfloat16" and kind != 0:
            return self._draw(kind, a, b, shape, "float32").astype("bfloat16")
        per = 2 if dt == "float64" else 4  # bf16 uniforms are the f32 stream, rounded
        n = int(math.prod(shape)) if shape else 1
        off = self._advance(n, per)
        if kind == 0 and _LAZY_RANDOM:
            # generated on first use; a reduction consuming it directly fuses
            # the generator into the reduction (sum, square_sum)
            return DeviceArray(shape, dt, lazy=("rand", 0, self._seed, off, float(a), float(b)))
        out = DeviceArray(shape, dt)
        driver().rand(kind, out.ptr, out.size, out.code, self._seed, off, float(a), float(b))
        return out

    def uniform(self, low=0.0, high=1.0, size=None, dtype="float64") -> DeviceArray:
        return self._draw(0, low, high, size, dtype)

    def randn(self, *shape, dtype="float64") -> DeviceArray:
        return self.normal(0.0, 1.0, shape or (1,), dtype)

    def standard_normal(self, size=None, dtype="float64") -> DeviceArray:
        return self.normal(0.0, 1.0, size, dtype)

    def normal(self, loc=0.0, scale=1.0, size=None, dtype="float64") -> DeviceArray:
        return self._draw(1, loc, scale, size, dtype)


def _shape_of(size) -> Shape:
    if size is None:
        return (1,)
    if is_integer(size):
        return (int(size),)
    if len(size) == 1 and isinstance(size[0], (tuple, list)):
        return tuple(int(s) for s in size[0])
    return tuple(int(s) for s in size)


class _RandomModule:
    """``bk.random`` — module-level functions on a default generator."""

    def __init__(self) -> None:
        self._gen: Optional[Generator] = None

    @property
    def gen(self) -> Generator:
        if self._gen is None:
            self._gen = Generator()
        return self._gen

    def seed(self, seed=None): self.gen.seed(seed)
    def default_rng(self, seed=None) -> Generator: return Generator(seed)
    def rand(self, *shape, dtype="float64"): return self.gen.rand(*shape, dtype=dtype)
    def randn(self, *shape, dtype="float64"): return self.gen.randn(*shape, dtype=dtype)
    def random(self, size=None, dtype="float64"): return self.gen.random(size, dtype)
    def uniform(self, low=0.0, high=1.0, size=None, dtype="float64"): return self.gen.uniform(low, high, size, dtype)
    def normal(self, loc=0.0, scale=1.0, size=None, dtype="float64"): return self.gen.normal(loc, scale, size, dtype)
    def standard_normal(self, size=None, dtype="float64"): return self.gen.standard_normal(size, dtype)


random = _RandomModule()


class Timer:
    """Device timing: HIP events (native) or synced wall clock (broker)."""

    def __enter__(self):
        self._tok = driver().timer_start()
        return self

    def __exit__(self, *exc):
        self.ms = driver().timer_stop(self._tok)
        return False
