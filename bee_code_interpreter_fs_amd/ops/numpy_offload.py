"""Opt-in numpy offload: unmodified numpy code on the sandbox's MI355X.

With offload on (``ExecuteRequest.numpy_offload``, or ``APP_NUMPY_OFFLOAD``
for every request) the sandbox patches ``numpy.random``'s legacy module
functions -- ``rand``, ``random`` / ``random_sample`` / ``ranf`` /
``sample``, ``uniform``, ``randn``, ``standard_normal``, ``normal`` -- and
the ``random`` / ``uniform`` / ``normal`` / ``standard_normal`` methods of
``numpy.random.default_rng()`` Generators, so a draw of at least ``BEE_NUMPY_OFFLOAD_MIN`` elements (default 2**20) returns
an :class:`OffloadArray`: a device array (Philox4x32-10 on the GPU,
``ops/array.py``) that numpy functions and operators dispatch on through
``__array_ufunc__`` / ``__array_function__`` (``ops/npinterop.py``).  The
reference's benchmark payload, byte for byte
(`/root/reference/examples/benchmark-numpy.py:15-28`)::

    large_array = numpy.random.rand(array_size)            # lazy device draw
    result = numpy.sum(numpy.square(large_array))          # one fused kernel

then runs as one Philox -> square -> reduce kernel.  This is the reference's
import-hook mechanism (`executor/sitecustomize.py:20-66` patches libraries on
import) applied to numpy; the reference itself never leaves the CPU.

What the user sees:

* values: the same distribution as numpy's, from a different generator
  (Philox, counter-based) -- ``numpy.random.seed(s)`` makes the device stream
  reproducible too, but it is not MT19937's stream;
* types: an OffloadArray is not an ``ndarray`` subclass; it has ``shape``,
  ``dtype`` (a numpy dtype), ``ndim``, ``size``, the reductions as methods,
  arithmetic operators, and every other ndarray attribute through a host copy;
* semantics: the first operation without a GPU kernel (indexing, slicing,
  printing, ``np.sort`` ...) copies the array to the host once and keeps it
  there -- from then on it is an ndarray in all but name (views alias it,
  in-place writes stick), with one ``HostFallbackWarning`` per function;
* reductions return numpy scalars (``numpy.float64`` / ``float32``) as numpy
  does; sums accumulate in f64 in a fixed order (deterministic).

Small draws (below the threshold) stay plain numpy: a kernel launch and a
device round trip cost more than numpy's own loop there.
"""

from __future__ import annotations

import functools
import math
import os
import sys
from typing import Optional

from . import npinterop
from ._lazy import np

MIN_ELEMENTS = int(os.environ.get("BEE_NUMPY_OFFLOAD_MIN", str(1 << 20)) or (1 << 20))


class _Residency:
    """Where one array's data lives: a device array, until the first host
    operation on it *or on any view of it* moves it to a host ndarray for
    good.  Views share their base's residency, so they keep aliasing one
    buffer on either side (a view moved to the host alone used to
    stop seeing writes through its base)."""

    __slots__ = ("dev", "host")

    def __init__(self, dev, host) -> None:
        self.dev, self.host = dev, host

    def to_host(self):
        if self.host is None:
            self.host = self.dev.numpy()
            self.dev = None
        return self.host


class OffloadArray:
    """A float64 / float32 numpy-like array resident on the GPU until an
    operation without a kernel moves it to the host for good."""

    __array_priority__ = 1000
    __slots__ = ("_res", "_vf", "_dview", "_hview", "__weakref__")
    __hash__ = None  # mutable, like ndarray

    def __init__(self, dev=None, host=None, res=None, vf=None) -> None:
        # vf: how this view derives from its base (reshape / T), applied to
        # the device array and to the host ndarray alike
        res = res if res is not None else _Residency(dev, host)
        object.__setattr__(self, "_res", res)
        object.__setattr__(self, "_vf", vf)
        object.__setattr__(self, "_dview", vf(res.dev) if (vf is not None and res.dev is not None) else None)
        object.__setattr__(self, "_hview", None)

    def _view(self, fn):
        """A view of this array sharing its residency (reshape / ravel / T)."""
        vf = self._vf
        return OffloadArray(res=self._res, vf=fn if vf is None else (lambda base: fn(vf(base))))

    # ---- residency -----------------------------------------------------------------
    @property
    def _dev(self):
        r = self._res
        if r.dev is None:
            return None
        return r.dev if self._vf is None else self._dview

    @property
    def _host(self):
        return None if self._res.host is None else self._h()

    @property
    def on_device(self) -> bool:
        return self._res.dev is not None

    def _h(self):
        """The host ndarray, downloading the base (once, for every view of
        it) and releasing the device copy."""
        base = self._res.to_host()
        if self._vf is None:
            return base
        if self._hview is None:
            object.__setattr__(self, "_hview", self._vf(base))
        return self._hview

    # ---- metadata (no transfer) ----------------------------------------------------
    @property
    def shape(self):
        d = self._dev
        return d.shape if d is not None else self._h().shape

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def size(self) -> int:
        d = self._dev
        return d.size if d is not None else self._h().size

    @property
    def dtype(self):
        d = self._dev
        return np.dtype(d.dtype) if d is not None else self._h().dtype

    @property
    def itemsize(self) -> int:
        return self.dtype.itemsize

    @property
    def nbytes(self) -> int:
        return self.size * self.itemsize

    # ---- numpy protocols -------------------------------------------------------------
    def __array__(self, dtype=None, copy=None):
        h = self._h()
        if dtype is not None and np.dtype(dtype) != h.dtype:
            return h.astype(dtype)
        return h.copy() if copy else h

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        return npinterop.array_ufunc(_BINDING, ufunc, method, inputs, kwargs)

    def __array_function__(self, func, types, args, kwargs):
        v = self._view_function(getattr(func, "__name__", ""), args, kwargs)
        if v is not None:
            return v
        return npinterop.array_function(_BINDING, func, types, args, kwargs)

    def _view_function(self, name, args, kwargs):
        """np.reshape / np.ravel / np.transpose of this device array: a view
        sharing its residency (not a new array), as numpy returns a view."""
        if not args or args[0] is not self or not self.on_device:
            return None
        kw = {k: v for k, v in kwargs.items() if npinterop._given(v)}
        if kw.pop("order", "C") not in ("C", None):
            return None
        if name == "reshape":
            if "newshape" in kw and "shape" not in kw:
                kw["shape"] = kw.pop("newshape")
            shape = args[1] if len(args) == 2 and "shape" not in kw else kw.pop("shape", None)
            if shape is None or kw or len(args) > 2:
                return None
            return self.reshape(shape)
        if name == "ravel" and len(args) == 1 and not kw:
            return self.ravel()
        if name == "transpose" and len(args) == 1 and not kw.get("axes") and self.ndim == 2:
            return self.T
        return None

    # ---- reductions and shape methods (device when resident) ------------------------
    def sum(self, axis=None, **kw):
        return np.sum(self, axis=axis, **kw)

    def mean(self, axis=None, **kw):
        return np.mean(self, axis=axis, **kw)

    def max(self, axis=None, **kw):
        return np.max(self, axis=axis, **kw)

    def min(self, axis=None, **kw):
        return np.min(self, axis=axis, **kw)

    def var(self, axis=None, **kw):
        return np.var(self, axis=axis, **kw)

    def std(self, axis=None, **kw):
        return np.std(self, axis=axis, **kw)

    def dot(self, other):
        return np.dot(self, other)

    def copy(self, order="C"):
        return np.copy(self) if order in ("C", "K", "A") else self._h().copy(order)

    def reshape(self, *shape, order="C"):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        if self.on_device and order in ("C", None):
            try:
                self._dev.reshape(shape)  # (validates the shape; device views share the buffer)
            except (ValueError, TypeError):
                return np.reshape(self, shape, order=order)
            return self._view(lambda base: base.reshape(shape))
        return self._h().reshape(shape, order=order)

    def ravel(self, order="C"):
        if self.on_device and order in ("C", None):
            return self._view(lambda base: base.reshape(-1))
        return self._h().ravel(order)

    def astype(self, dtype, *args, **kwargs):
        dt = np.dtype(dtype)
        if self._dev is not None and not args and not kwargs and dt.name in ("float32", "float64"):
            return OffloadArray(self._dev.astype(dt.name))
        return self._h().astype(dtype, *args, **kwargs)

    def item(self, *args):
        if not args and self.size == 1 and self._dev is not None:
            return self._dev.item()
        return self._h().item(*args)

    def __getattr__(self, name):
        # anything else an ndarray has: on the host copy
        if name.startswith("__") or name in ("_res", "_vf", "_dview", "_hview"):
            raise AttributeError(name)
        if self.on_device:
            npinterop.warn_fallback(f"ndarray.{name}")
        return getattr(self._h(), name)

    def __setattr__(self, name, value):
        if name in ("shape", "dtype", "strides", "flags", "data", "real", "imag", "flat"):
            setattr(self._h(), name, value)
        else:
            object.__setattr__(self, name, value)

    # ---- Python protocols ----------------------------------------------------------
    def __len__(self):
        if not self.shape:
            raise TypeError("len() of unsized object")
        return self.shape[0]

    def __iter__(self):
        return iter(self._h())

    def __getitem__(self, key):
        return self._h()[key]

    def __setitem__(self, key, value):
        self._h()[key] = np.asarray(value) if isinstance(value, OffloadArray) else value

    def __contains__(self, v):
        return v in self._h()

    def __repr__(self):
        return repr(self._h())

    def __str__(self):
        return str(self._h())

    def __format__(self, spec):
        return format(self._h(), spec)

    def __bool__(self):
        if self.size != 1:
            raise ValueError("The truth value of an array with more than one element is ambiguous. "
                             "Use a.any() or a.all()")
        return bool(self.item())

    def __float__(self):
        return float(self.item())

    def __int__(self):
        return int(self.item())

    def __index__(self):
        return self._h().__index__()

    def __copy__(self):
        return self.copy()

    def __deepcopy__(self, memo):
        return self.copy()

    def __reduce__(self):
        return (_host_array, (self._h(),))

    # operators: through the ufuncs, so the dispatch above decides where they run
    def __add__(self, o): return np.add(self, o)
    def __radd__(self, o): return np.add(o, self)
    def __iadd__(self, o): return np.add(self, o, out=(self,))
    def __sub__(self, o): return np.subtract(self, o)
    def __rsub__(self, o): return np.subtract(o, self)
    def __isub__(self, o): return np.subtract(self, o, out=(self,))
    def __mul__(self, o): return np.multiply(self, o)
    def __rmul__(self, o): return np.multiply(o, self)
    def __imul__(self, o): return np.multiply(self, o, out=(self,))
    def __truediv__(self, o): return np.true_divide(self, o)
    def __rtruediv__(self, o): return np.true_divide(o, self)
    def __itruediv__(self, o): return np.true_divide(self, o, out=(self,))
    def __floordiv__(self, o): return np.floor_divide(self, o)
    def __rfloordiv__(self, o): return np.floor_divide(o, self)
    def __mod__(self, o): return np.remainder(self, o)
    def __rmod__(self, o): return np.remainder(o, self)
    def __pow__(self, o): return np.power(self, o)
    def __rpow__(self, o): return np.power(o, self)
    def __ipow__(self, o): return np.power(self, o, out=(self,))
    def __matmul__(self, o): return np.matmul(self, o)
    def __rmatmul__(self, o): return np.matmul(o, self)
    def __neg__(self): return np.negative(self)
    def __pos__(self): return self.copy()
    def __abs__(self): return np.absolute(self)
    def __lt__(self, o): return np.less(self, o)
    def __le__(self, o): return np.less_equal(self, o)
    def __gt__(self, o): return np.greater(self, o)
    def __ge__(self, o): return np.greater_equal(self, o)
    def __eq__(self, o): return np.equal(self, o)
    def __ne__(self, o): return np.not_equal(self, o)

    @property
    def T(self):
        if self.on_device and self.ndim == 2:
            return self._view(lambda base: base.T)
        return self._h().T


def _host_array(a):
    return a


def _dev_of(x):
    return x._dev if isinstance(x, OffloadArray) else None


def _host_of(x):
    return x._h()


_BINDING = npinterop.Binding(dev=_dev_of, box=lambda d: OffloadArray(d), host=_host_of,
                             is_mine=lambda x: isinstance(x, OffloadArray))


# ---- numpy.random patches -------------------------------------------------------------

_GEN: list = []  # the sandbox's device generator, created on first use


def _gen():
    if not _GEN:
        from .array import Generator

        _GEN.append(Generator())  # seeded from os.urandom, like numpy's global state per process
    return _GEN[0]


def _count(shape) -> Optional[int]:
    """Elements of a size argument made of plain integers, else None."""
    if shape is None:
        return None
    if isinstance(shape, (int, np.integer)) and not isinstance(shape, bool):
        return int(shape)
    if isinstance(shape, (tuple, list)) and all(isinstance(s, (int, np.integer)) and not isinstance(s, bool)
                                                 for s in shape):
        return math.prod(int(s) for s in shape)
    return None


def _scalar(v) -> bool:
    return isinstance(v, (int, float, np.floating, np.integer)) and not isinstance(v, bool)


def _big(shape) -> bool:
    n = _count(shape)
    return n is not None and n >= MIN_ELEMENTS and all(int(s) >= 0 for s in
                                                      ((shape,) if not isinstance(shape, (tuple, list)) else shape))


def _shape(shape):
    return (int(shape),) if not isinstance(shape, (tuple, list)) else tuple(int(s) for s in shape)


def _wrap_rand(orig):
    @functools.wraps(orig)
    def rand(*shape):
        if shape and _big(tuple(shape)):
            return OffloadArray(_gen().uniform(0.0, 1.0, _shape(tuple(shape))))
        return orig(*shape)

    return rand


def _wrap_randn(orig):
    @functools.wraps(orig)
    def randn(*shape):
        if shape and _big(tuple(shape)):
            return OffloadArray(_gen().normal(0.0, 1.0, _shape(tuple(shape))))
        return orig(*shape)

    return randn


def _wrap_sample(orig):
    @functools.wraps(orig)
    def random_sample(size=None):
        if _big(size):
            return OffloadArray(_gen().uniform(0.0, 1.0, _shape(size)))
        return orig(size)

    return random_sample


def _wrap_uniform(orig):
    @functools.wraps(orig)
    def uniform(low=0.0, high=1.0, size=None):
        if _big(size) and _scalar(low) and _scalar(high) and math.isfinite(float(low)) and math.isfinite(float(high)):
            return OffloadArray(_gen().uniform(float(low), float(high), _shape(size)))
        return orig(low, high, size)

    return uniform


def _wrap_normal(orig):
    @functools.wraps(orig)
    def normal(loc=0.0, scale=1.0, size=None):
        if _big(size) and _scalar(loc) and _scalar(scale) and float(scale) >= 0.0 and math.isfinite(float(loc)):
            return OffloadArray(_gen().normal(float(loc), float(scale), _shape(size)))
        return orig(loc, scale, size)

    return normal


def _wrap_standard_normal(orig):
    @functools.wraps(orig)
    def standard_normal(size=None):
        if _big(size):
            return OffloadArray(_gen().normal(0.0, 1.0, _shape(size)))
        return orig(size)

    return standard_normal


def _wrap_seed(orig):
    @functools.wraps(orig)
    def seed(seed=None):
        orig(seed)
        # the device stream follows: the same seed, the same draws (Philox,
        # keyed by the seed's integer; numpy's MT19937 stream is not reproduced)
        if seed is None:
            _gen().seed(None)
        elif isinstance(seed, (int, np.integer)):
            _gen().seed(int(seed))
        else:
            arr = np.asarray(seed, dtype=np.uint64).ravel()
            _gen().seed(int.from_bytes(arr.tobytes()[:8].ljust(8, b"\0"), "little") ^ (len(arr) << 56))

    return seed


def _generator_class():
    """numpy.random.Generator with its large float draws on the device: what
    the patched ``default_rng`` returns.  A subclass, so ``isinstance(rng,
    np.random.Generator)`` (scipy's ``check_random_state`` and the like)
    holds, and every method without a device kernel (integers, choice,
    shuffle, ...) is numpy's own on the same bit generator."""
    if _GENCLS:
        return _GENCLS[0]

    class Generator(np.random.Generator):
        def __init__(self, bit_generator):
            super().__init__(bit_generator)
            from .array import Generator as DeviceGenerator

            # the device stream is keyed by the seed sequence: default_rng(s)
            # twice gives the same device draws (Philox, not PCG64's stream)
            state = bit_generator.seed_seq.generate_state(2, np.uint64) if hasattr(bit_generator, "seed_seq") \
                else np.frombuffer(os.urandom(16), np.uint64)
            self._bee_dev = DeviceGenerator(int(state[0]) ^ (int(state[1]) << 1))

        def _ok(self, size, dtype=np.float64, out=None):
            return out is None and _big(size) and np.dtype(dtype).name in ("float32", "float64")

        def random(self, size=None, dtype=np.float64, out=None):
            if self._ok(size, dtype, out):
                return OffloadArray(self._bee_dev.uniform(0.0, 1.0, _shape(size), np.dtype(dtype).name))
            return super().random(size, dtype, out)

        def uniform(self, low=0.0, high=1.0, size=None):
            if self._ok(size) and _scalar(low) and _scalar(high) and math.isfinite(float(low)) and \
                    math.isfinite(float(high)):
                return OffloadArray(self._bee_dev.uniform(float(low), float(high), _shape(size)))
            return super().uniform(low, high, size)

        def standard_normal(self, size=None, dtype=np.float64, out=None):
            if self._ok(size, dtype, out):
                return OffloadArray(self._bee_dev.normal(0.0, 1.0, _shape(size), np.dtype(dtype).name))
            return super().standard_normal(size, dtype, out)

        def normal(self, loc=0.0, scale=1.0, size=None):
            if self._ok(size) and _scalar(loc) and _scalar(scale) and float(scale) >= 0.0 and math.isfinite(float(loc)):
                return OffloadArray(self._bee_dev.normal(float(loc), float(scale), _shape(size)))
            return super().normal(loc, scale, size)

    Generator.__module__ = "numpy.random"
    _GENCLS.append(Generator)
    return Generator


_GENCLS: list = []


def _wrap_default_rng(orig):
    @functools.wraps(orig)
    def default_rng(seed=None):
        rng = orig(seed)
        if seed is not None and isinstance(seed, np.random.Generator):
            return rng  # numpy returns a Generator passed in unaltered
        return _generator_class()(rng.bit_generator)

    return default_rng


_WRAPPERS = {
    "rand": _wrap_rand,
    "randn": _wrap_randn,
    "random": _wrap_sample,
    "random_sample": _wrap_sample,
    "ranf": _wrap_sample,
    "sample": _wrap_sample,
    "uniform": _wrap_uniform,
    "normal": _wrap_normal,
    "standard_normal": _wrap_standard_normal,
    "seed": _wrap_seed,
    "default_rng": _wrap_default_rng,
}


def patch_numpy_random(npr, setter=setattr) -> None:
    """Wrap ``npr``'s legacy draw functions (``setter``: how attributes are
    set -- tests pass pytest's monkeypatch.setattr so numpy is restored)."""
    if getattr(npr, "_bee_offload", False):
        return
    for name, wrap in _WRAPPERS.items():
        orig = getattr(npr, name, None)
        if orig is not None:
            setter(npr, name, wrap(orig))
    setter(npr, "_bee_offload", True)


def install() -> None:
    """Turn the offload on in this process: now if numpy.random is loaded,
    else when it is imported (runtime/sandbox_patches.py's import hook)."""
    from ..runtime import sandbox_patches

    sandbox_patches.add_patch("numpy.random", patch_numpy_random)


def installed() -> bool:
    npr = sys.modules.get("numpy.random")
    return bool(npr is not None and getattr(npr, "_bee_offload", False))
