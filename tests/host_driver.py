"""A numpy model of the beekern kernel driver, for CPU tests of the layers
above the kernels (``ops/array.py``, the numpy protocols in
``ops/npinterop.py``, the offload in ``ops/numpy_offload.py``).

It implements the driver interface of ``ops/driver.py`` (NativeDriver /
BrokerDriver) op by op, with the kernels' semantics: the Philox uniform
streams bit for bit (tests/philox_ref.py), f64 accumulation for reductions,
bf16 storage as RNE-rounded f32 bits, GEMMs on bf16 operands with f32
results.  Tests install it explicitly (``use_host_driver``); the package
never selects it -- on a GPU box the real kernels run or the ops fail.
"""

from __future__ import annotations

import bisect

import numpy as np

from .philox_ref import uniform_f32, uniform_f64

_NP = {0: np.float32, 1: np.float64, 2: np.uint16}
_SIZE = {0: 4, 1: 8, 2: 2}


def _bf16_bits(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    out = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(a)
    if nan.any():
        out[nan] = 0x7FC0
    return out


def _bf16_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


class HostDriver:
    name = "host-model"

    def __init__(self) -> None:
        self.device = 0
        self._bases: list = []
        self._mem: dict = {}
        self._next = 1 << 20
        self.launches: list = []  # (op name, ...) in order: what the kernels would have run

    def init(self, device: int, lazy: bool = False) -> None:
        self.device = device

    # ---- memory -----------------------------------------------------------------------
    def malloc(self, nbytes: int) -> int:
        h = self._next
        self._next += ((max(int(nbytes), 1) + 255) // 256) * 256 + 256
        self._mem[h] = np.zeros(max(int(nbytes), 1), np.uint8)
        bisect.insort(self._bases, h)
        return h

    def free(self, h: int) -> None:
        if h in self._mem:
            del self._mem[h]
            self._bases.remove(h)

    def _at(self, p: int, nbytes: int) -> np.ndarray:
        i = bisect.bisect_right(self._bases, p) - 1
        base = self._bases[i]
        buf = self._mem[base]
        off = p - base
        assert 0 <= off and off + nbytes <= buf.size, "out of bounds"
        return buf[off: off + nbytes]

    def _view(self, p: int, n: int, dt: int) -> np.ndarray:
        return self._at(p, n * _SIZE[dt]).view(_NP[dt])

    def _load(self, p: int, n: int, dt: int) -> np.ndarray:
        v = self._view(p, n, dt)
        return _bf16_f32(v).astype(np.float64) if dt == 2 else v.astype(np.float64)

    def _store(self, p: int, vals: np.ndarray, dt: int) -> None:
        v = self._view(p, vals.size, dt)
        v[...] = _bf16_bits(vals.astype(np.float32)) if dt == 2 else vals.astype(_NP[dt])

    def h2d(self, h: int, host: np.ndarray, offset: int = 0) -> None:
        raw = np.ascontiguousarray(host).view(np.uint8).ravel()
        self._at(h + offset, raw.size)[...] = raw

    def d2h(self, h: int, host: np.ndarray, offset: int = 0) -> None:
        self.launches.append(("d2h", host.nbytes))
        host.view(np.uint8).ravel()[...] = self._at(h + offset, host.nbytes)

    def copy(self, dst: int, src: int, nbytes: int) -> None:
        self._at(dst, nbytes)[...] = self._at(src, nbytes)

    def fill(self, y: int, nbytes: int, pattern: int, width: int) -> None:
        dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[width]
        self._at(y, nbytes).view(dt)[...] = pattern

    # ---- kernels ----------------------------------------------------------------------
    def _draw(self, kind, n, dt, seed, off, a, b):
        if kind == 0:
            if dt == 1:
                return uniform_f64(n, seed, off, a, b)
            return uniform_f32(n, seed, off, a, b).astype(np.float64)
        rng = np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFFFFFFFFFF, off]))  # (default_rng may be patched)
        return rng.normal(a, b, n)

    def rand(self, kind, h, n, dt, seed, off, a, b) -> None:
        self.launches.append(("rand", kind, n))
        self._store(h, self._draw(kind, n, dt, seed, off, a, b), dt)

    _UNARY = [np.square, np.abs, np.negative, np.sqrt, np.exp, np.log, lambda x: np.maximum(x, 0), np.sin, np.cos,
              np.tanh, lambda x: 1 / (1 + np.exp(-x)), lambda x: x]

    def unary(self, op, dt, x, y, n) -> None:
        self.launches.append(("unary", op, n))
        with np.errstate(all="ignore"):
            self._store(y, self._UNARY[op](self._load(x, n, dt)), dt)

    _BINARY = [np.add, np.subtract, np.multiply, np.divide, np.maximum, np.minimum, np.power]

    def binary(self, op, dt, mode, a, b, sc, y, n) -> None:
        self.launches.append(("binary", op, n))
        x = self._load(a, n, dt)
        with np.errstate(all="ignore"):
            if mode == 0:
                r = self._BINARY[op](x, self._load(b, n, dt))
            elif mode == 1:
                r = self._BINARY[op](x, sc)
            else:
                r = self._BINARY[op](sc, x)
        self._store(y, r, dt)

    def cast(self, s, d, x, y, n) -> None:
        self.launches.append(("cast", s, d, n))
        self._store(y, self._load(x, n, s), d)

    def _reduce_vals(self, op, a, b):
        with np.errstate(all="ignore"):
            if op == 0:
                return float(a.sum())
            if op == 1:
                return float((a * a).sum())
            if op == 2:
                return float(np.abs(a).sum())
            if op == 3:
                return float(a.max())
            if op == 4:
                return float(a.min())
            if op == 5:
                return float((a * b).sum())
            return float(np.abs(a - b).max())

    def reduce(self, op, dt, a, b, n) -> float:
        self.launches.append(("reduce", op, n))
        return self._reduce_vals(op, self._load(a, n, dt), self._load(b, n, dt) if b else None)

    def rand_reduce(self, op, dt, n, seed, off, lo, hi) -> float:
        self.launches.append(("rand_reduce", op, n))
        return self._reduce_vals(op, self._draw(0, n, dt, seed, off, lo, hi), None)

    def reduce_axis(self, op, dt, x, y, rows, cols, ld, axis) -> None:
        self.launches.append(("reduce_axis", op, axis))
        m = self._load(x, rows * ld, dt).reshape(rows, ld)[:, :cols]
        r = m.sum(axis=axis)
        if op == 1:
            r = r / (rows if axis == 0 else cols)
        self._store(y, r, 1 if dt == 1 else 0)

    def transpose(self, src, dst, rows, cols, ldi, ldo, src_dtype=2, dst_dtype=2) -> None:
        self.launches.append(("transpose", rows, cols))
        m = self._load(src, rows * ldi, src_dtype).reshape(rows, ldi)[:, :cols]
        out = self._load(dst, cols * ldo, dst_dtype).reshape(cols, ldo)
        out[:, :rows] = m.T.astype(np.float32).astype(np.float64) if dst_dtype == 2 else m.T
        self._store(dst, out.ravel(), dst_dtype)

    def gemm(self, A, Bt, C, M, N, K, lda, ldb, ldc, alpha, beta, odt) -> None:
        self.launches.append(("gemm", M, N, K))
        a = self._load(A, M * lda, 2).reshape(M, lda)[:, :K]
        bt = self._load(Bt, N * ldb, 2).reshape(N, ldb)[:, :K]
        self._gemm_out(a @ bt.T, C, M, N, ldc, alpha, beta, odt)

    def gemm_nn(self, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, odt) -> None:
        self.launches.append(("gemm_nn", M, N, K))
        a = self._load(A, M * lda, 2).reshape(M, lda)[:, :K]
        b = self._load(B, K * ldb, 2).reshape(K, ldb)[:, :N]
        self._gemm_out(a @ b, C, M, N, ldc, alpha, beta, odt)

    def gemm_fp(self, dt, ta, tb, A, B, C, M, N, K, lda, ldb, ldc) -> None:
        self.launches.append(("gemm_fp", dt, M, N, K, bool(ta), bool(tb)))
        a = self._load(A, (K if ta else M) * lda, dt).reshape(-1, lda)[:, : (M if ta else K)]
        b = self._load(B, (N if tb else K) * ldb, dt).reshape(-1, ldb)[:, : (K if tb else N)]
        a = a.T if ta else a
        b = b.T if tb else b
        np_dt = _NP[dt]
        prod = a.astype(np_dt) @ b.astype(np_dt)  # numpy's own product in the dtype
        c = self._load(C, M * ldc, dt).reshape(M, ldc)
        c[:, :N] = prod
        self._store(C, c.ravel(), dt)

    def gemm_f32x6(self, ta, tb, A, B, C, M, N, K, lda, ldb, ldc, W, ws_bytes) -> None:
        self.launches.append(("gemm_f32x6", M, N, K, bool(ta), bool(tb)))
        assert ws_bytes == 256 + 12 * ((K + 63) // 64 * 64) * (M + N)
        self._load(W, ws_bytes // 2, 2)  # (the workspace exists and is that large)
        self.gemm_fp(0, ta, tb, A, B, C, M, N, K, lda, ldb, ldc)
        self.launches.pop()  # (the inner gemm_fp's own entry)

    def _gemm_out(self, prod, C, M, N, ldc, alpha, beta, odt):
        c = self._load(C, M * ldc, odt).reshape(M, ldc)
        c[:, :N] = alpha * prod.astype(np.float32) + (beta * c[:, :N] if beta else 0.0)
        self._store(C, c.ravel(), odt)

    def sync(self) -> None:
        return None

    def memory_stats(self) -> dict:
        used = sum(b.size for b in self._mem.values())
        return {"in_use": used, "cached": 0, "peak": used, "quota": 0}

    def set_quota(self, q: int) -> None:
        return None

    def note_quota(self, q: int) -> None:
        return None

    def empty_cache(self) -> None:
        return None

    def device_info(self) -> dict:
        return {"arch": "host-model", "compute_units": 0, "total_bytes": 0, "free_bytes": 0, "clock_khz": 0,
                "lds_bytes_per_cu": 0}

    def timer_start(self):
        return 0.0

    def timer_stop(self, tok) -> float:
        return 0.0


def use_host_driver(monkeypatch) -> HostDriver:
    """Point beekern at a fresh HostDriver for one test."""
    import sys

    A = sys.modules["bee_code_interpreter_fs_amd.ops.array"]  # (the package exports a function named `array`)
    drv = HostDriver()
    monkeypatch.setattr(A, "_driver", drv)
    return drv
