"""numpy on the MI355X: the numpy protocols of beekern arrays
(ops/npinterop.py) and the opt-in numpy offload (ops/numpy_offload.py) on
the real kernels -- in this process (native driver) and through the service
(a "min" sandbox on the kernel broker).  CPU twin: test_numpy_offload_cpu.py.
"""

import os
import tempfile

import numpy as np
import pytest

from .harness import ServiceHarness, ensure_native_executor

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE_PAYLOAD = os.path.join(ROOT, "examples", "benchmark_numpy_reference.py")
N8 = 10**8
SIGMA = (N8 * 4 / 45) ** 0.5


def test_numpy_functions_on_device_arrays_match_numpy(gpu):
    rng = np.random.default_rng(5)
    h = rng.standard_normal((512, 384))
    x = gpu.asarray(h)
    assert np.sum(x) == pytest.approx(h.sum(), rel=1e-12, abs=1e-9)
    assert np.mean(x) == pytest.approx(h.mean(), rel=1e-12, abs=1e-12)
    assert np.max(x) == h.max() and np.min(x) == h.min()
    np.testing.assert_allclose(np.sum(x, axis=0).numpy(), h.sum(axis=0), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(np.mean(x, axis=1).numpy(), h.mean(axis=1), rtol=1e-12, atol=1e-12)
    assert np.sum(np.square(x)) == pytest.approx((h * h).sum(), rel=1e-12)
    assert np.var(x) == pytest.approx(h.var(), rel=1e-10) and np.std(x) == pytest.approx(h.std(), rel=1e-10)
    assert np.linalg.norm(x) == pytest.approx(np.linalg.norm(h), rel=1e-12)
    v = gpu.asarray(h[0])
    assert np.dot(v, v) == pytest.approx(h[0] @ h[0], rel=1e-12)
    y = np.add(np.multiply(x, 2.0), 1.0)
    assert isinstance(y, gpu.DeviceArray)
    np.testing.assert_allclose(y.numpy(), 2.0 * h + 1.0, rtol=1e-15)
    np.testing.assert_allclose(np.exp(np.negative(np.absolute(x))).numpy(), np.exp(-np.abs(h)), rtol=1e-12)


def test_reference_payload_in_process_under_offload(gpu, monkeypatch):
    """The reference's benchmark-numpy payload, verbatim, with numpy.random
    patched in this process: 1e8 draws reduced by one fused kernel on the
    GPU; Result within 6 sigma of n/3 and a numpy.float64 as numpy returns."""
    import contextlib
    import io

    from bee_code_interpreter_fs_amd.ops import numpy_offload

    monkeypatch.setattr(numpy_offload, "_GEN", [])
    numpy_offload.patch_numpy_random(np.random, setter=lambda o, k, v: monkeypatch.setattr(o, k, v, raising=False))
    buf = io.StringIO()
    ns = {"__name__": "__main__"}
    with contextlib.redirect_stdout(buf):
        exec(compile(open(REFERENCE_PAYLOAD).read(), REFERENCE_PAYLOAD, "exec"), ns)
    assert isinstance(ns["result"], np.float64)
    assert abs(float(ns["result"]) - N8 / 3) < 6 * SIGMA
    assert float(buf.getvalue().split("Execution Time:")[1].split()[0]) < 1.0


@pytest.fixture(scope="module")
def osvc():
    ensure_native_executor()
    h = ServiceHarness(tempfile.mkdtemp(prefix="bee-offload-"), gpu_ids=[0], workers_per_gpu_target=1,
                       default_timeout=120.0)
    h.start()
    yield h
    h.stop()


def test_reference_payload_through_the_service_with_offload(osvc):
    """Unmodified numpy code, Execute(numpy_offload=True): the draw and the
    square-sum run on the sandbox's GPU through the kernel broker."""
    src = open(REFERENCE_PAYLOAD).read()
    r = osvc.call(osvc.ctx.code_executor.execute(source_code=src, numpy_offload=True, timeout=120), timeout=300)
    assert r.exit_code == 0, r.stderr
    assert abs(float(r.stdout.split("Result:")[1].split()[0]) - N8 / 3) < 6 * SIGMA
    t = float(r.stdout.split("Execution Time:")[1].split()[0])
    assert t < 0.5, r.stdout  # numpy on the CPU takes ~1 s of this
    assert "HostFallbackWarning" not in r.stderr, r.stderr


def test_offloaded_arrays_fall_back_correctly_in_a_sandbox(osvc):
    code = (
        "import numpy as np\n"
        "np.random.seed(7)\n"
        "x = np.random.rand(2_000_000)\n"
        "a = float(np.sum(x))\n"
        "np.random.seed(7)\n"
        "y = np.random.rand(2_000_000)\n"
        "assert float(np.sum(y)) == a\n"
        "m = np.mean(x * 2.0 + 1.0)\n"
        "top = np.sort(x)[-1]\n"          # no kernel: host copy, numpy's answer
        "assert top == np.max(x) and type(x).__name__ == 'OffloadArray'\n"
        "print(round(m, 2), round(a / 2_000_000, 2))\n"
    )
    r = osvc.call(osvc.ctx.code_executor.execute(source_code=code, numpy_offload=True, timeout=120), timeout=300)
    assert r.exit_code == 0, r.stderr
    assert r.stdout.split() == ["2.0", "0.5"], r.stdout
    assert "HostFallbackWarning" in r.stderr and "sort" in r.stderr
