"""CPU test of beekern's matmul operand lowering (ops/array.py:matmul): which
device ops a call issues for each kind of ``b``, recorded by a fake driver.
The kernels themselves are covered on the GPU (test_kernels_gpu.py)."""

import importlib

import numpy as np
import pytest

from bee_code_interpreter_fs_amd.ops._native import DTYPE_CODES

# the module (the package re-exports a function named ``array``)
arr = importlib.import_module("bee_code_interpreter_fs_amd.ops.array")


class FakeDriver:
    def __init__(self, name):
        self.name = name
        self.device = 0
        self.calls = []
        self._next = 0x1000

    def malloc(self, n):
        self._next += (n + 255) // 256 * 256 + 256
        return self._next

    def free(self, p):
        pass

    def h2d(self, h, host, offset=0):
        pass

    def cast(self, s, d, x, y, n):
        self.calls.append(("cast", s, d, n))

    def transpose(self, src, dst, rows, cols, ldi, ldo, src_dtype=2, dst_dtype=2):
        self.calls.append(("transpose", rows, cols, src_dtype))

    def gemm(self, a, bt, c, M, N, K, lda, ldb, ldc, alpha, beta, odt):
        self.calls.append(("gemm", M, N, K))


@pytest.fixture(params=["native", "broker"])
def fake(request, monkeypatch):
    d = FakeDriver(request.param)
    monkeypatch.setattr(arr, "_driver", d)
    return d


def _ops(d):
    return [c[0] for c in d.calls]


def test_bf16_b_transposed_view_is_used_as_is(fake):
    a = arr.DeviceArray((64, 32), "bfloat16")
    bt = arr.DeviceArray((48, 32), "bfloat16")
    arr.matmul(a, bt.T)
    assert _ops(fake) == ["gemm"]
    assert fake.calls[-1] == ("gemm", 64, 48, 32)


def test_bf16_row_major_b_is_transposed_once(fake):
    arr.matmul(arr.DeviceArray((64, 32), "bfloat16"), arr.DeviceArray((32, 48), "bfloat16"))
    assert fake.calls == [("transpose", 32, 48, DTYPE_CODES["bfloat16"]), ("gemm", 64, 48, 32)]


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_wide_row_major_b_is_converted_in_the_transpose(fake, dtype):
    arr.matmul(arr.DeviceArray((64, 32), "bfloat16"), arr.DeviceArray((32, 48), dtype))
    assert fake.calls == [("transpose", 32, 48, DTYPE_CODES[dtype]), ("gemm", 64, 48, 32)]


def test_wide_transposed_view_is_only_converted(fake):
    bt = arr.DeviceArray((48, 32), "float32")
    arr.matmul(arr.DeviceArray((64, 32), "bfloat16"), bt.T)
    assert fake.calls == [("cast", DTYPE_CODES["float32"], DTYPE_CODES["bfloat16"], 48 * 32), ("gemm", 64, 48, 32)]


def test_unaligned_wide_b_falls_back_to_cast_then_transpose(fake):
    arr.matmul(arr.DeviceArray((64, 30), "bfloat16"), arr.DeviceArray((30, 44), "float64"))
    assert _ops(fake) == ["cast", "transpose", "gemm"]
    assert fake.calls[1] == ("transpose", 30, 44, DTYPE_CODES["bfloat16"])


def test_wide_a_is_cast_first(fake):
    arr.matmul(arr.DeviceArray((64, 32), "float64"), arr.DeviceArray((48, 32), "bfloat16").T)
    assert _ops(fake) == ["cast", "gemm"]


def test_shape_mismatch_raises(fake):
    with pytest.raises(ValueError):
        arr.matmul(arr.DeviceArray((64, 32), "bfloat16"), arr.DeviceArray((31, 48), "bfloat16"))
    assert fake.calls == []


def test_host_operand_is_uploaded(fake):
    arr.matmul(np.zeros((16, 8), np.float32), arr.DeviceArray((8, 24), "bfloat16"))
    assert _ops(fake) == ["cast", "transpose", "gemm"]


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_wide_transposed_view_materialises_on_device(fake, dtype):
    x = arr.DeviceArray((24, 40), dtype)
    x.T._materialize()
    code = DTYPE_CODES[dtype]
    assert fake.calls == [("transpose", 24, 40, code)]


class FakeNNDriver(FakeDriver):
    def gemm_nn(self, a, b, c, M, N, K, lda, ldb, ldc, alpha, beta, odt):
        self.calls.append(("gemm_nn", M, N, K))


@pytest.mark.parametrize("mode,M,expect", [
    ("auto", 4096, ["gemm_nn"]),               # transpose pass ~15% of the GEMM at M=4096: read B in place
    ("auto", 8192, ["transpose", "gemm"]),     # ~7% at M=8192: the faster TN kernel after the pass
    ("1", 8192, ["gemm_nn"]),
    ("0", 4096, ["transpose", "gemm"]),
])
def test_row_major_bf16_b_kernel_choice(monkeypatch, mode, M, expect):
    d = FakeNNDriver("broker")
    monkeypatch.setattr(arr, "_driver", d)
    monkeypatch.setattr(arr, "_GEMM_NN", mode)
    arr.matmul(arr.DeviceArray((M, 1024), "bfloat16"), arr.DeviceArray((1024, 4096), "bfloat16"))
    assert _ops(d) == expect


def test_row_major_bf16_b_off_tile_shape_is_transposed(monkeypatch):
    d = FakeNNDriver("broker")
    monkeypatch.setattr(arr, "_driver", d)
    monkeypatch.setattr(arr, "_GEMM_NN", "auto")
    arr.matmul(arr.DeviceArray((4000, 1024), "bfloat16"), arr.DeviceArray((1024, 4096), "bfloat16"))
    assert _ops(d) == ["transpose", "gemm"]
