"""numpy on device arrays, on CPU: the dispatch of ``ops/npinterop.py``
(NEP 13 / NEP 18) and the opt-in numpy offload of ``ops/numpy_offload.py``,
over a numpy model of the kernel driver (tests/host_driver.py) that records
which kernels would have run.  The same behaviour on the MI355X kernels is
in tests/test_offload_gpu.py."""

import os
import warnings

import numpy as np
import pytest

from bee_code_interpreter_fs_amd import ops
from bee_code_interpreter_fs_amd.ops import npinterop, numpy_offload
from bee_code_interpreter_fs_amd.ops.numpy_offload import OffloadArray

from .host_driver import use_host_driver

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 16  # above the offload threshold set below, small for the host model


@pytest.fixture
def drv(monkeypatch):
    d = use_host_driver(monkeypatch)
    monkeypatch.setattr(npinterop, "_WARNED", set())
    return d


@pytest.fixture
def offload(drv, monkeypatch):
    """numpy.random patched for one test (monkeypatch restores numpy)."""
    monkeypatch.setattr(numpy_offload, "MIN_ELEMENTS", 1 << 12)
    monkeypatch.setattr(numpy_offload, "_GEN", [])
    numpy_offload.patch_numpy_random(np.random, setter=lambda o, k, v: monkeypatch.setattr(o, k, v, raising=False))
    return drv


def kernels(drv):
    return [op[0] for op in drv.launches]


# ---- DeviceArray (the explicit beekern API) ---------------------------------------------

def test_np_sum_of_device_array_runs_on_the_reduction_kernel(drv):
    x = ops.asarray(np.linspace(0.0, 1.0, 1001))
    drv.launches.clear()
    s = np.sum(x)
    assert kernels(drv) == ["reduce"], drv.launches  # no d2h of the array: the kernel's scalar only
    assert isinstance(s, np.float64) and s == pytest.approx(500.5)
    assert np.mean(x) == pytest.approx(0.5) and np.max(x) == 1.0 and np.min(x) == 0.0


def test_np_square_then_sum_is_the_fused_square_sum(drv):
    x = ops.random.default_rng(3).random(N)  # lazy draw
    drv.launches.clear()
    v = np.sum(np.square(x))
    assert kernels(drv) == ["rand_reduce"], drv.launches  # neither the draw nor x**2 materialised
    from .philox_ref import uniform_f64

    assert v == pytest.approx(float(np.square(uniform_f64(N, 3)).sum()), rel=1e-12)


def test_ufuncs_and_scalars_stay_on_device(drv):
    h = np.linspace(0.5, 2.0, 4096)
    x = ops.asarray(h)
    for got, want in [(np.add(x, 1.5), h + 1.5), (np.multiply(2.0, x), 2.0 * h), (np.subtract(1.0, x), 1.0 - h),
                      (np.divide(x, x), h / h), (np.sqrt(x), np.sqrt(h)), (np.exp(x), np.exp(h)),
                      (np.maximum(x, 1.0), np.maximum(h, 1.0)), (np.power(x, 3.0), h ** 3.0),
                      (np.negative(x), -h), (np.absolute(np.negative(x)), h)]:
        assert isinstance(got, ops.DeviceArray), type(got)
        np.testing.assert_allclose(got.numpy(), want, rtol=1e-12)
    assert np.add.reduce(x) == pytest.approx(h.sum())
    assert np.maximum.reduce(x) == h.max()


def test_axis_reductions_and_1d_dot(drv):
    h = np.arange(12.0).reshape(3, 4)
    x = ops.asarray(h)
    np.testing.assert_allclose(np.sum(x, axis=0).numpy(), h.sum(axis=0))
    np.testing.assert_allclose(np.mean(x, axis=1).numpy(), h.mean(axis=1))
    a, b = ops.asarray(np.arange(5.0)), ops.asarray(np.ones(5))
    assert np.dot(a, b) == 10.0
    assert np.linalg.norm(a) == pytest.approx(np.linalg.norm(np.arange(5.0)))
    assert np.var(a) == pytest.approx(np.var(np.arange(5.0))) and np.std(a, ddof=1) == pytest.approx(
        np.std(np.arange(5.0), ddof=1))
    assert np.shape(x) == (3, 4) and np.ndim(x) == 2 and np.size(x) == 12


def test_float32_keeps_numpy_types_and_promotion(drv):
    h = np.linspace(0, 1, 100, dtype=np.float32)
    x = ops.asarray(h)
    s = np.sum(x)
    assert isinstance(s, np.float32)
    y = np.multiply(x, 2.0)  # Python scalar: weak, stays f32 on the device
    assert isinstance(y, ops.DeviceArray) and y.dtype == "float32"
    with pytest.warns(npinterop.HostFallbackWarning):
        z = np.multiply(x, np.float64(2.0))  # a float64 scalar promotes (NEP 50): numpy's answer, on the host
    assert isinstance(z, np.ndarray) and z.dtype == np.float64


def test_unsupported_calls_fall_back_with_one_warning(drv):
    h = np.array([3.0, 1.0, 2.0])
    x = ops.asarray(h)
    with pytest.warns(npinterop.HostFallbackWarning, match="sort"):
        r = np.sort(x)
    np.testing.assert_array_equal(r, np.sort(h))
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        np.sort(x)  # warned once per function per process
    with pytest.warns(npinterop.HostFallbackWarning):
        np.testing.assert_array_equal(np.cumsum(x), np.cumsum(h))


def test_matmul_of_f64_arrays_runs_at_numpy_precision(drv, monkeypatch):
    """f64 products go to the f64 MFMA GEMM (gemm_fp), never the bf16 one."""
    rng = np.random.default_rng(0)
    a_h, b_h = rng.standard_normal((64, 32)), rng.standard_normal((32, 16))
    a, b = ops.asarray(a_h), ops.asarray(b_h)
    drv.launches.clear()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no host fallback
        c = np.matmul(a, b)
    assert isinstance(c, ops.DeviceArray) and c.dtype == "float64" and c.shape == (64, 16)
    assert [k[:2] for k in drv.launches] == [("gemm_fp", 1)], drv.launches
    np.testing.assert_allclose(c.numpy(), a_h @ b_h, rtol=1e-12)
    monkeypatch.setenv("BEE_NUMPY_OFFLOAD_MATMUL", "bf16")
    c2 = np.matmul(a, b)  # opted in: the bf16 MFMA GEMM
    assert isinstance(c2, ops.DeviceArray) and "gemm," in ",".join(kernels(drv)) + ","
    np.testing.assert_allclose(c2.numpy(), a_h @ b_h, atol=0.3)


def test_large_f32_matmul_takes_the_split_bf16_product(drv, monkeypatch):
    """f32 products above 2^33 multiply-adds (M, N >= 256) run as the six-piece
    bf16 split (gemm_f32x6) with an exactly-sized workspace; small ones, f64,
    BEE_GEMM_F32X6=0 and a quota with no room for the workspace stay on the
    f32 / f64 MFMA (gemm_fp)."""
    import importlib

    arr = importlib.import_module("bee_code_interpreter_fs_amd.ops.array")  # (ops.array is the function)
    rng = np.random.default_rng(5)
    a_h = rng.standard_normal((2048, 2560)).astype(np.float32)
    b_h = rng.standard_normal((2048, 2560)).astype(np.float32)
    a, b = ops.asarray(a_h), ops.asarray(b_h)
    drv.launches.clear()
    c = np.matmul(a, b.T)  # 2048 x 2048 x 2560 > 2^33
    assert kernels(drv) == ["gemm_f32x6"] and drv.launches[0][-2:] == (False, True), drv.launches
    assert c.dtype == "float32"
    np.testing.assert_allclose(c.numpy(), a_h @ b_h.T, rtol=1e-4, atol=1e-3)
    assert arr.f32x6_workspace_bytes(1024, 1024, 1000) == 256 + 12 * 1024 * 2048
    drv.launches.clear()
    np.matmul(ops.asarray(a_h[:200]), b.T)  # M < 256
    np.matmul(ops.asarray(a_h[:, :2048]), ops.asarray(b_h[:, :2048].T))  # 2^33: not above
    np.matmul(ops.asarray(a_h.astype(np.float64)), ops.asarray(b_h.T.astype(np.float64)))
    monkeypatch.setattr(arr, "_F32X6", "0")
    np.matmul(a, b.T)
    assert kernels(drv) == ["gemm_fp"] * 4, drv.launches
    monkeypatch.setattr(arr, "_F32X6", "auto")

    real_malloc = drv.malloc

    def tight(nbytes):  # the workspace does not fit the quota
        if nbytes >= arr.f32x6_workspace_bytes(2048, 2048, 2560):
            raise ops.QuotaExceeded("no room")
        return real_malloc(nbytes)

    monkeypatch.setattr(drv, "malloc", tight)
    drv.launches.clear()
    np.matmul(a, b.T)
    assert kernels(drv) == ["gemm_fp"], drv.launches


def test_matmul_dtypes_views_vectors_and_host_operands(drv):
    rng = np.random.default_rng(1)
    a_h = rng.standard_normal((48, 40))
    a = ops.asarray(a_h)
    # a .T view is read in place: one GEMM with the transposed-A flag, no transpose pass
    drv.launches.clear()
    g = np.dot(a.T, a)
    assert kernels(drv) == ["gemm_fp"] and drv.launches[0][-2:] == (True, False), drv.launches
    np.testing.assert_allclose(g.numpy(), a_h.T @ a_h, rtol=1e-12, atol=1e-12)
    # 1-D operands: numpy's vector rules
    v_h = rng.standard_normal(40)
    r = a @ ops.asarray(v_h)
    assert r.shape == (48,)
    np.testing.assert_allclose(r.numpy(), a_h @ v_h, rtol=1e-12)
    # a host ndarray operand is uploaded once; the result stays on the device
    h = rng.standard_normal((40, 8))
    drv.launches.clear()
    r2 = np.matmul(a, h)
    assert isinstance(r2, ops.DeviceArray) and kernels(drv) == ["gemm_fp"]
    np.testing.assert_allclose(r2.numpy(), a_h @ h, rtol=1e-12)
    # f32 stays f32; f32 with a host int64 operand promotes to f64, as numpy does
    a32 = ops.asarray(a_h.astype(np.float32))
    c32 = np.matmul(a32, ops.asarray(h.astype(np.float32)))
    assert c32.dtype == "float32" and drv.launches[-1][1] == 0
    np.testing.assert_allclose(c32.numpy(), a_h.astype(np.float32) @ h.astype(np.float32), rtol=1e-5, atol=1e-5)
    ints = np.arange(40 * 3).reshape(40, 3)
    c64 = np.matmul(a32, ints)
    assert c64.dtype == "float64" and c64.shape == (48, 3)
    np.testing.assert_allclose(c64.numpy(), a_h.astype(np.float32).astype(np.float64) @ ints, rtol=1e-12)
    # batched (3-D) and mismatched shapes: numpy's answer / error, on the host
    with pytest.warns(npinterop.HostFallbackWarning):
        np.testing.assert_allclose(np.matmul(a, np.ones((2, 40, 3))), a_h @ np.ones((2, 40, 3)))
    with pytest.raises(ValueError):
        np.matmul(a, np.ones((39, 3)))


def test_reshape_keywords_follow_numpy(drv):
    """np.reshape(x, newshape=...) kept its shape out (a flat
    array came back) and copy=True returned an aliasing view."""
    x = ops.asarray(np.arange(12.0))
    r = np.reshape(x, newshape=(3, 4))
    assert r.shape == (3, 4)
    assert np.reshape(x, (4, 3)).shape == (4, 3) and np.reshape(x, shape=(2, 6)).shape == (2, 6)
    with pytest.warns(npinterop.HostFallbackWarning):
        c = np.reshape(x, (3, 4), copy=True)  # numpy's copy, not a device view
    c[0, 0] = 99.0
    assert float(x.numpy()[0]) == 0.0


def test_out_argument_writes_in_place(drv):
    x = ops.asarray(np.ones(1000))
    y = x.reshape(10, 100)  # shares the buffer
    r = np.add(x, 1.0, out=(x,))
    assert r is x and float(np.sum(y)) == 2000.0  # the view sees the write


# ---- the offload (patched numpy.random) ---------------------------------------------------

def test_offloaded_draw_is_a_lazy_device_array(offload):
    x = np.random.rand(N)
    assert isinstance(x, OffloadArray) and x.on_device
    assert x.shape == (N,) and x.dtype == np.float64 and x.ndim == 1 and x.size == N and len(x) == N
    assert offload.launches == []  # nothing ran yet: the draw is lazy
    small = np.random.rand(10)
    assert type(small) is np.ndarray  # below the threshold: numpy


def test_reference_payload_lowers_to_one_fused_kernel(offload):
    """The reference's payload (examples/benchmark_numpy_reference.py, the
    reference file verbatim) with its size scaled down for the host model:
    one Philox -> square -> reduce launch, a numpy.float64 result."""
    src = open(os.path.join(ROOT, "examples", "benchmark_numpy_reference.py")).read()
    assert "array_size = 10**8" in src
    ns = {"__name__": "__main__"}
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        exec(compile(src.replace("10**8", str(N)), "payload", "exec"), ns)
    assert kernels(offload) == ["rand_reduce"], offload.launches
    assert isinstance(ns["result"], np.float64)
    value = float(buf.getvalue().split("Result:")[1].split()[0])
    assert abs(value - N / 3) < 6 * (N * 4 / 45) ** 0.5


def test_seed_makes_the_device_stream_reproducible(offload):
    np.random.seed(1234)
    a = float(np.sum(np.random.rand(N)))
    b = float(np.sum(np.random.rand(N)))
    np.random.seed(1234)
    assert float(np.sum(np.random.rand(N))) == a and a != b


def test_host_fallback_keeps_numpy_semantics(offload):
    x = np.random.uniform(-1.0, 1.0, N)
    s_dev = float(np.sum(x))
    with pytest.warns(npinterop.HostFallbackWarning):
        first = x.argmax()  # no kernel: the array moves to the host, once
    assert not x.on_device
    h = np.asarray(x)
    assert first == h.argmax() and abs(float(np.sum(x)) - s_dev) < 1e-9 * N
    v = x[:10]  # a view of the host copy
    x[0] = 42.0  # writes stick and views alias it, as an ndarray's would
    assert v[0] == 42.0 and np.max(x) == 42.0
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # host-resident now: plain numpy, no more warnings
        assert (x > 0.5).dtype == bool and (x > 0.5).shape == (N,) and np.cumsum(x).shape == (N,)
    assert "array(" in repr(x[:3]) or isinstance(x[:3], np.ndarray)


def test_operators_inplace_and_statistics(offload):
    x = np.random.rand(N)
    y = x * 2.0 + 1.0
    assert isinstance(y, OffloadArray) and y.on_device
    x += 1.0
    assert x.on_device and float(np.min(x)) >= 1.0 and float(np.max(x)) < 2.0
    z = np.random.standard_normal(N)
    assert abs(float(np.mean(z))) < 0.05 and abs(float(np.std(z)) - 1.0) < 0.05
    m = np.random.normal(3.0, 2.0, (256, 256))
    assert m.shape == (256, 256) and abs(float(m.mean()) - 3.0) < 0.05
    col = np.sum(m, axis=0)
    assert isinstance(col, OffloadArray) and col.shape == (256,)
    assert x.astype(np.float32).dtype == np.float32


def test_offloaded_matrices_multiply_on_the_device(offload):
    """``np.random.rand(n, n) @ np.random.rand(n, n)``: both draws offloaded,
    the product on the f64 GEMM, an OffloadArray back."""
    a = np.random.rand(128, 64)
    b = np.random.rand(64, 96)
    c = a @ b
    assert isinstance(c, OffloadArray) and c.on_device and c.shape == (128, 96) and c.dtype == np.float64
    assert "gemm_fp" in kernels(offload)
    d = np.dot(a.T, np.ones(128))  # a host vector operand: uploaded, the result stays on the device
    assert isinstance(d, OffloadArray) and d.on_device and d.shape == (64,)
    a_h = np.asarray(a)  # (the first host operation moves an offloaded array to the host for good)
    np.testing.assert_allclose(np.asarray(c), a_h @ np.asarray(b), rtol=1e-12)
    np.testing.assert_allclose(np.asarray(d), a_h.sum(axis=0), rtol=1e-12)


def test_payload_without_offload_is_plain_numpy(drv):
    assert type(np.random.rand(N)) is np.ndarray


# ---- the request field through the service to the sandbox ----------------------------------

PROBE = ("import numpy as np\n"
         "print(getattr(np.random, '_bee_offload', False), type(np.random.rand(3)).__name__)\n")


def test_numpy_offload_field_reaches_the_sandbox(tmp_path):
    """``numpy_offload`` (gRPC field 104, HTTP ``numpy_offload``) travels
    front-end -> executor job -> pooled sandbox, which patches numpy.random
    for that run only; without it numpy is untouched.  (A virtual GPU slot:
    this machine has no GPU, and the probe's draw is below the threshold.)"""
    import grpc
    import httpx

    from bee_code_interpreter_fs_amd.models import proto as pb

    from .harness import ServiceHarness, ensure_native_executor

    ensure_native_executor()
    h = ServiceHarness(str(tmp_path), gpu_ids=[0], broker_enabled=False, worker_warm_gpu=False,
                       workers_per_gpu_target=1)
    h.start()
    try:
        with grpc.insecure_channel(h.grpc_target) as ch:
            stub = pb.CodeInterpreterServiceStub(ch)
            on = stub.Execute(pb.ExecuteRequest(source_code=PROBE, numpy_offload=True), timeout=120)
            off = stub.Execute(pb.ExecuteRequest(source_code=PROBE), timeout=120)
        assert (on.exit_code, on.stdout) == (0, "True ndarray\n"), on.stderr
        assert (off.exit_code, off.stdout) == (0, "False ndarray\n"), off.stderr
        r = httpx.post(h.http_base + "/v1/execute", json={"source_code": PROBE, "numpy_offload": True}, timeout=120)
        assert r.status_code == 200 and r.json()["stdout"] == "True ndarray\n", r.text
    finally:
        h.stop()


def test_views_share_residency_with_their_base(offload):
    """a reshape / ravel / T view moved to the host alone
    stopped aliasing its base.  Now the first host operation on any view
    moves the base, and every view aliases the one host buffer."""
    a = np.random.rand(64 * 64)
    b = a.reshape(64, 64)
    c = np.reshape(a, (32, 128))
    t = b.T
    assert all(isinstance(v, OffloadArray) and v.on_device for v in (b, c, t))
    b[0, 1] = 5.0  # the base and every view move to the host together
    assert not a.on_device and not c.on_device and not t.on_device
    assert a[1] == 5.0 and c[0, 1] == 5.0 and t[1, 0] == 5.0
    a[2] = 7.0
    assert b[0, 2] == 7.0 and np.ravel(a)[2] == 7.0


def test_default_rng_draws_are_offloaded(offload):
    rng = np.random.default_rng(42)
    assert isinstance(rng, np.random.Generator)
    x = rng.random(N)
    assert isinstance(x, OffloadArray) and x.on_device
    y = rng.standard_normal((128, 64))
    assert isinstance(y, OffloadArray) and y.shape == (128, 64)
    assert abs(float(np.mean(y))) < 0.05
    assert type(rng.random(10)) is np.ndarray  # small: numpy
    assert rng.integers(0, 10, 5).shape == (5,)  # no kernel: numpy's own, same bit generator
    same = float(np.sum(np.random.default_rng(42).random(N)))
    assert same == float(np.sum(np.random.default_rng(42).random(N)))  # seeded: reproducible
    assert np.random.default_rng(rng) is rng
    f32 = rng.random(N, dtype=np.float32)
    assert f32.dtype == np.float32
