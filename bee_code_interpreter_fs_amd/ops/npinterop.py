"""numpy's dispatch protocols for beekern arrays (NEP 13 ``__array_ufunc__``,
NEP 18 ``__array_function__``).

A numpy call on a device array runs on the gfx950 kernels when one computes
what numpy would (same dtype rules, same shape):

* ufuncs: square, negative, absolute, sqrt, exp, log, sin, cos, tanh, add,
  subtract, multiply, divide, maximum, minimum, power -- elementwise kernels
  (``ops/array.py`` ``_unary`` / ``_binary``); ``np.square`` stays lazy, so
  ``np.sum(np.square(x))`` is the fused one-pass square-sum;
* ufunc reductions ``np.add.reduce`` / ``np.maximum.reduce`` /
  ``np.minimum.reduce``;
* functions: ``sum`` / ``mean`` (whole array or one axis of a 2-D array),
  ``max`` / ``min`` / ``amax`` / ``amin``, ``dot`` of 1-D vectors, ``var`` /
  ``std`` (two passes, as numpy), ``linalg.norm`` (fused square-sum),
  ``copy`` / ``reshape`` / ``ravel``, and the metadata functions
  ``shape`` / ``ndim`` / ``size``;
* ``matmul`` / ``dot`` / ``@`` of 1-D and 2-D operands: f32 / f64 on the
  full-precision MFMA GEMM in numpy's result dtype (``ops/array.py``
  ``matmul_fp``, ``csrc/kernels/gemm_fp.hip``; ``.T`` views read in place),
  bf16 on the bf16 MFMA GEMM.  A host ndarray operand of a product with a
  device array is uploaded once and the result stays on the device
  (``BEE_NUMPY_OFFLOAD_MATMUL=bf16`` rounds f32 / f64 products to the bf16
  GEMM instead, as before).

Everything else copies the operands to the host (``__array__``) and runs
numpy there, with one ``HostFallbackWarning`` per function per process
(``BEE_OFFLOAD_WARN=0`` silences it).  ``np.sum(device_array)`` used to
take that copy silently for every call (the class had only ``__array__``).

The reference has no GPU path at all; this is the in-sandbox half of the
north star's "sandboxed code calls the HIP kernels in place of numpy"
(BASELINE.json), opt-in through ``ops/numpy_offload.py``.
"""

from __future__ import annotations

import math
import os
import warnings
from typing import Any, Callable, Optional

from ._lazy import np


def _array_module():
    # (the package exports a function named `array`: reach the module itself)
    import importlib

    return importlib.import_module(__package__ + ".array")


class HostFallbackWarning(UserWarning):
    """A numpy call on a device array ran on the host (operands copied)."""


_WARNED: set = set()


def warn_fallback(what: str) -> None:
    if what in _WARNED or os.environ.get("BEE_OFFLOAD_WARN", "1") == "0":
        return
    _WARNED.add(what)
    warnings.warn(f"beekern: numpy.{what} has no GPU kernel for these operands; they were copied to the host",
                  HostFallbackWarning, stacklevel=4)


_UNARY = {"square": "square", "negative": "negative", "absolute": "abs", "sqrt": "sqrt", "exp": "exp", "log": "log",
          "sin": "sin", "cos": "cos", "tanh": "tanh"}
_BINARY = {"add": "add", "subtract": "subtract", "multiply": "multiply", "divide": "divide",
           "true_divide": "divide", "maximum": "maximum", "minimum": "minimum", "power": "power"}
_REDUCE = {"add": "sum", "maximum": "amax", "minimum": "amin"}


class Binding:
    """How one array class plugs into the dispatch: ``dev(x)`` -> the
    device array behind ``x`` (or None if ``x`` is not device-resident),
    ``box(d)`` -> a result device array as the caller's class, ``host(x)`` ->
    the ndarray for a host fallback, ``scalar(v, dtype)`` -> a reduction's
    result as numpy would type it."""

    def __init__(self, dev: Callable, box: Callable, host: Callable, is_mine: Callable) -> None:
        self.dev, self.box, self.host, self.is_mine = dev, box, host, is_mine


def _weak_scalar_ok(s, dtype_name: str) -> bool:
    """A scalar operand keeps the array's dtype (numpy 2 / NEP 50): Python
    int / float / bool are weak; a numpy scalar must not promote."""
    if isinstance(s, (np.floating, np.integer, np.bool_)):  # (np.float64 is also a Python float)
        if dtype_name == "bfloat16":
            return False
        return np.result_type(np.dtype(dtype_name), s) == np.dtype(dtype_name)
    if isinstance(s, (bool, int, float)):
        return not isinstance(s, int) or abs(s) < 2**53
    return False


def _as_result_scalar(v, dtype_name: str):
    """numpy types a full reduction by the array's dtype (f32 -> float32)."""
    if dtype_name == "float32":
        return np.float32(v)
    return np.float64(v)


def _host_args(b: Binding, obj):
    if b.is_mine(obj):
        return b.host(obj)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_host_args(b, o) for o in obj)
    if isinstance(obj, dict):
        return {k: _host_args(b, v) for k, v in obj.items()}
    return obj


def _any_on_device(b: Binding, objs) -> bool:
    """Whether a host fallback moves anything off the device (arrays already
    on the host -- an offloaded array after its first host operation -- are
    plain numpy from then on: no warning)."""
    for o in objs:
        if b.dev(o) is not None:
            return True
        if isinstance(o, (list, tuple)) and _any_on_device(b, o):
            return True
    return False


_FP = ("float32", "float64")


def _matmul(b: Binding, A, x, y, name: str = "matmul"):
    """The device result of numpy's ``matmul`` / ``dot`` of ``x`` and ``y``
    (numpy's dtype rules and 1-D semantics), or None for a host fallback.

    One operand may be a host ndarray (or list) when the other is on the
    device: it is uploaded once -- a product with a device array is worth one
    host-to-device copy of the other operand -- and the result stays on the
    device.  N-D (batched) operands, integer results and shape errors go to
    numpy on the host (which raises numpy's own error for the last)."""
    dx, dy = b.dev(x), b.dev(y)
    if dx is None and dy is None:
        return None
    if (dx is None and b.is_mine(x)) or (dy is None and b.is_mine(y)):
        return None  # a host-resident offload array: everything stays on the host
    if "bfloat16" in (getattr(dx, "dtype", None), getattr(dy, "dtype", None)):
        if dx is None or dy is None or dx.dtype != dy.dtype or dx.ndim != 2 or dy.ndim != 2 or \
                dx.shape[1] != dy.shape[0]:
            return None
        return A.matmul(dx, dy)

    def np_dtype(obj, d):
        if d is not None:
            return np.dtype(d.dtype)
        h = np.asarray(obj)
        return h.dtype if h.dtype.kind in "biuf" and h.ndim in (1, 2) and h.size else None

    tx, ty = np_dtype(x, dx), np_dtype(y, dy)
    if tx is None or ty is None:
        return None
    rt = np.result_type(tx, ty)
    if rt.name not in _FP:
        return None
    shapes = [d.shape if d is not None else np.shape(o) for o, d in ((x, dx), (y, dy))]
    if any(len(s) not in (1, 2) for s in shapes):
        return None
    if name == "dot" and len(shapes[0]) == 1 and len(shapes[1]) == 1:
        return None  # (1-D . 1-D is the reduction path)
    kx = shapes[0][-1]
    ky = shapes[1][0]
    if kx != ky:
        return None
    if dx is None:
        dx = A.asarray(np.asarray(x), rt.name)
    if dy is None:
        dy = A.asarray(np.asarray(y), rt.name)
    if os.environ.get("BEE_NUMPY_OFFLOAD_MATMUL", "") == "bf16" and dx.ndim == 2 and dy.ndim == 2:
        return A.matmul(dx, dy, out_dtype="float32").astype(rt.name)
    return A.matmul_fp(dx, dy)


def array_ufunc(b: Binding, ufunc, method: str, inputs, kwargs):
    A = _array_module()

    out = kwargs.get("out")
    extra = {k for k in kwargs if k != "out"}
    name = ufunc.__name__
    res = _try_ufunc(b, A, ufunc, name, method, inputs, kwargs, extra)
    if res is not None:
        if out is not None:
            target = b.dev(out[0])
            A.driver().unary(A._UNARY["copy"], target.code, res.ptr, target.ptr, target.size)
            return out[0]
        return b.box(res) if isinstance(res, A.DeviceArray) else res
    if _any_on_device(b, inputs):
        warn_fallback(name if method == "__call__" else f"{name}.{method}")
    return getattr(ufunc, method)(*_host_args(b, inputs), **_host_args(b, kwargs))


def _try_ufunc(b, A, ufunc, name, method, inputs, kwargs, extra) -> Optional[Any]:
    """The GPU result (DeviceArray or numpy scalar), or None for a host fallback."""
    out = kwargs.get("out")
    if method == "__call__":
        if extra - {"dtype"}:
            return None
        if name == "matmul":
            if len(inputs) != 2 or out is not None or kwargs.get("dtype") is not None:
                return None
            return _matmul(b, A, inputs[0], inputs[1])
        devs = [b.dev(x) for x in inputs]
        arrays = [d for d in devs if d is not None]
        if not arrays or any(b.is_mine(x) and d is None for x, d in zip(inputs, devs)):
            return None  # a host-resident operand: everything stays on the host
        dt = arrays[0].dtype
        if kwargs.get("dtype") is not None and np.dtype(kwargs["dtype"]).name != dt:
            return None
        if any(d.dtype != dt for d in arrays):
            return None
        if out is not None:
            if len(out) != 1 or b.dev(out[0]) is None:
                return None
            o = b.dev(out[0])
            if o.dtype != dt or o.shape != arrays[0].shape or o._transposed:
                return None
            o._materialize()  # (a lazy draw gets its buffer: the result is written into it)
        if name in _UNARY and len(inputs) == 1:
            x = devs[0]
            return A.square(x) if name == "square" else A._unary(_UNARY[name], x)
        if name in _BINARY and len(inputs) == 2:
            x, y = devs
            if x is not None and y is not None:
                if x.shape != y.shape:
                    return None
                if name == "multiply" and inputs[0] is inputs[1]:
                    return A.square(x)
                return A._binary(_BINARY[name], x, y)
            arr, s, rev = (x, inputs[1], False) if x is not None else (y, inputs[0], True)
            if not _weak_scalar_ok(s, dt):
                return None
            if name == "power" and not rev and float(s) == 2.0:
                return A.square(arr)
            return A._binary(_BINARY[name], arr, float(s), reversed_=rev)
        return None
    if method == "reduce" and name in _REDUCE and len(inputs) == 1 and out is None:
        if extra - {"axis", "dtype"}:
            return None
        x = b.dev(inputs[0])
        if x is None or (kwargs.get("dtype") is not None and np.dtype(kwargs["dtype"]).name != x.dtype):
            return None
        axis = kwargs.get("axis", 0)
        if axis is None or (x.ndim == 1 and axis in (0, -1)):
            return _full_reduce(A, _REDUCE[name], x)
        if name == "add" and x.ndim == 2 and axis in (0, 1, -1, -2):
            return A.sum(x, axis=axis)
        return None
    return None


def _full_reduce(A, what: str, x):
    v = A.sum(x) if what == "sum" else A.amax(x) if what == "amax" else A.amin(x)
    return _as_result_scalar(v, x.dtype)


_NOVALUE_NAMES = ("_NoValue", "_NoValueType")


def _given(v) -> bool:
    """An optional argument the caller actually passed (numpy forwards its
    ``np._NoValue`` sentinel for the ones left out)."""
    return v is not None and type(v).__name__ not in _NOVALUE_NAMES


def _kw_only(kwargs, allowed) -> bool:
    return all(k in allowed or not _given(v) or (k == "keepdims" and v is False) for k, v in kwargs.items())


def _bind(func_name: str, args, kwargs, params):
    """Positional + keyword arguments of ``func_name`` as a dict (the numpy
    signature's leading parameters ``params``); None if they do not fit."""
    if len(args) > len(params):
        return None
    got = dict(zip(params, args))
    for k, v in kwargs.items():
        if k in got:
            return None
        got[k] = v
    return got


def array_function(b: Binding, func, types, args, kwargs):
    A = _array_module()

    name = getattr(func, "__name__", str(func))
    mod = getattr(func, "__module__", "") or ""
    res = _try_function(b, A, name, mod, args, kwargs)
    if res is not _NO:
        return res
    if _any_on_device(b, args) or _any_on_device(b, tuple(kwargs.values())):
        warn_fallback(name if not mod.endswith("linalg") else f"linalg.{name}")
    return func(*_host_args(b, args), **_host_args(b, kwargs))


_NO = object()


def _try_function(b, A, name, mod, args, kwargs):
    if name in ("shape", "ndim", "size") and args and b.dev(args[0]) is not None and len(args) + len(kwargs) == 1:
        d = b.dev(args[0])
        return {"shape": d.shape, "ndim": d.ndim, "size": d.size}[name]
    if name in ("sum", "mean"):
        got = _bind(name, args, kwargs, ("a", "axis", "dtype", "out", "keepdims"))
        if got is None or not _kw_only(got, {"a", "axis"}):
            return _NO
        x = b.dev(got["a"])
        if x is None:
            return _NO
        axis = got.get("axis")
        if axis is None or (x.ndim == 1 and axis in (0, -1)):
            v = A.sum(x) if name == "sum" else A.mean(x)
            return _as_result_scalar(v, x.dtype)
        if x.ndim == 2 and isinstance(axis, int) and axis in (0, 1, -1, -2):
            return b.box(A.sum(x, axis=axis) if name == "sum" else A.mean(x, axis=axis))
        return _NO
    if name in ("max", "min", "amax", "amin"):
        got = _bind(name, args, kwargs, ("a", "axis", "out", "keepdims"))
        if got is None or not _kw_only(got, {"a"}):
            return _NO
        x = b.dev(got["a"])
        if x is None:
            return _NO
        return _full_reduce(A, "amax" if name in ("max", "amax") else "amin", x)
    if name in ("var", "std"):
        got = _bind(name, args, kwargs, ("a", "axis", "dtype", "out", "ddof", "keepdims"))
        if got is None or not _kw_only(got, {"a", "ddof"}):
            return _NO
        x = b.dev(got["a"])
        ddof = got.get("ddof", 0) if _given(got.get("ddof")) else 0
        if x is None or x.dtype == "bfloat16" or not isinstance(ddof, (int, float)):
            return _NO
        n = x.size
        if n - ddof <= 0:
            return _NO
        m = float(A.mean(x))
        v = float(A.square_sum(A._binary("subtract", x, m))) / (n - ddof)  # two passes, as numpy
        return _as_result_scalar(math.sqrt(v) if name == "std" else v, x.dtype)
    if name == "norm" and mod.endswith("linalg"):
        got = _bind(name, args, kwargs, ("x", "ord", "axis", "keepdims"))
        if got is None or not _kw_only(got, {"x"}):
            return _NO
        x = b.dev(got["x"])
        if x is None:
            return _NO
        return _as_result_scalar(math.sqrt(float(A.square_sum(x))), x.dtype)
    if name in ("dot", "vdot", "inner"):
        if len(args) != 2 or not _kw_only(kwargs, ()):
            return _NO
        x, y = b.dev(args[0]), b.dev(args[1])
        if x is not None and y is not None and x.ndim == 1 and y.ndim == 1 and x.shape == y.shape and \
                x.dtype == y.dtype:
            return _as_result_scalar(A.dot(x, y), x.dtype)
        if name == "dot":
            r = _matmul(b, A, args[0], args[1], "dot")
            return _NO if r is None else b.box(r)
        return _NO
    if name == "copy" and len(args) == 1 and not kwargs:
        x = b.dev(args[0])
        return _NO if x is None else b.box(x.copy())
    if name in ("reshape", "ravel"):
        params = ("a", "shape") if name == "reshape" else ("a",)
        kw = dict(kwargs)
        if name == "reshape" and "newshape" in kw:  # numpy < 2.1's name, deprecated but still accepted
            if "shape" in kw or len(args) > 1:
                return _NO
            kw["shape"] = kw.pop("newshape")
        got = _bind(name, args, kw, params + ("order",))
        # anything else (copy=..., unknown keywords): numpy decides, on the host
        if got is None or set(got) - set(params) - {"order"} or got.get("order", "C") not in ("C", None):
            return _NO
        if name == "reshape" and "shape" not in got:
            return _NO
        x = b.dev(got["a"])
        if x is None:
            return _NO
        shape = got.get("shape", -1) if name == "reshape" else -1
        try:
            return b.box(x.reshape(shape))
        except (ValueError, TypeError):
            return _NO
    return _NO
