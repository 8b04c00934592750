"""ctypes binding of ``libbeekern.so`` (csrc/kernels, built for gfx950).

Loading rules (SURVEY.md §0 dev-box facts, §7.3 item 4):

* torch-ROCm bundles its own ``libamdhip64.so.7``; the kernel library links
  the same SONAME.  Importing torch *first* makes the dynamic loader reuse
  torch's copy, so one HIP runtime serves both torch and beekern in a process.
  Sandboxes pre-import torch in the zygote, so this costs nothing there.
* the library is looked up in-tree (``ops/lib/libbeekern.so``) or at
  ``$BEE_KERNEL_LIB``; a missing library is a hard error on a GPU host —
  there is no silent CPU fallback for kernels that claim to run on MI355X.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_LIB_NAME = "libbeekern.so"
_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


class BeekernError(RuntimeError):
    pass


class QuotaExceeded(BeekernError, MemoryError):
    pass


STATUS = {
    0: "ok",
    1: "bad argument",
    2: "launch failed",
    3: "out of device memory",
    4: "HBM quota exceeded",
    5: "device not initialized",
}

# dtype codes shared with csrc/kernels/bk_common.hpp
DTYPE_CODES = {"float32": 0, "float64": 1, "bfloat16": 2, "float16": 3, "int32": 4, "int64": 5}
DTYPE_SIZES = {"float32": 4, "float64": 8, "bfloat16": 2, "float16": 2, "int32": 4, "int64": 8}


def library_path() -> str:
    env = os.environ.get("BEE_KERNEL_LIB")
    if env:
        return env
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", _LIB_NAME)


def _preload_torch_runtime() -> None:
    if os.environ.get("BEE_BEEKERN_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
    except Exception:
        pass


def _declare(lib: ctypes.CDLL) -> None:
    c_int, c_i64, c_u64, c_vp, c_d, c_f = (
        ctypes.c_int,
        ctypes.c_int64,
        ctypes.c_uint64,
        ctypes.c_void_p,
        ctypes.c_double,
        ctypes.c_float,
    )
    sig = {
        "bk_version": ([], c_int),
        "bk_last_error": ([], ctypes.c_char_p),
        "bk_init": ([c_int], c_int),
        "bk_device": ([], c_int),
        "bk_set_quota": ([c_i64], c_int),
        "bk_quota": ([], c_i64),
        "bk_malloc": ([ctypes.POINTER(c_vp), c_i64], c_int),
        "bk_free": ([c_vp], c_int),
        "bk_empty_cache": ([], c_int),
        "bk_memory_stats": ([ctypes.POINTER(c_i64)], c_int),
        "bk_memcpy": ([c_vp, c_vp, c_i64, c_int, c_vp], c_int),
        "bk_memcpy_async": ([c_vp, c_vp, c_i64, c_int, c_vp], c_int),
        "bk_sync": ([c_vp], c_int),
        "bk_preload": ([c_vp], c_int),
        "bk_device_info": ([ctypes.POINTER(c_i64), ctypes.c_char_p, c_int], c_int),
        "bk_event_pair_create": ([ctypes.POINTER(c_vp), ctypes.POINTER(c_vp)], c_int),
        "bk_event_record": ([c_vp, c_vp], c_int),
        "bk_event_elapsed_ms": ([c_vp, c_vp], c_f),
        "bk_event_destroy": ([c_vp], c_int),
        "bk_rand_uniform": ([c_vp, c_i64, c_int, c_u64, c_u64, c_d, c_d, c_vp], c_int),
        "bk_rand_normal": ([c_vp, c_i64, c_int, c_u64, c_u64, c_d, c_d, c_vp], c_int),
        "bk_unary": ([c_int, c_int, c_vp, c_vp, c_i64, c_vp], c_int),
        "bk_binary": ([c_int, c_int, c_int, c_vp, c_vp, c_d, c_vp, c_i64, c_vp], c_int),
        "bk_cast": ([c_int, c_int, c_vp, c_vp, c_i64, c_vp], c_int),
        "bk_fill": ([c_vp, c_i64, c_u64, c_int, c_vp], c_int),
        "bk_reduce_workspace_bytes": ([], c_int),
        "bk_reduce": ([c_int, c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp], c_int),
        "bk_rand_reduce": ([c_int, c_int, c_i64, c_u64, c_u64, c_d, c_d, c_vp, c_vp, c_vp], c_int),
        "bk_reduce_axis_workspace_bytes": ([], c_i64),
        "bk_reduce_workspace_init": ([c_vp, c_vp], c_int),
        "bk_reduce_axis_workspace_init": ([c_vp, c_vp], c_int),
        "bk_reduce_axis": ([c_int, c_int, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp], c_int),
        "bk_gemm_bf16_fast_ok": ([c_int, c_int, c_int, c_int, c_int], c_int),
        "bk_gemm_bf16_tn": (
            [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_f, c_int, c_vp],
            c_int,
        ),
        "bk_gemm_bf16_tn_variant": (
            [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_f, c_int, c_int, c_vp],
            c_int,
        ),
        "bk_gemm_bf16_pick": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int], c_int),
        "bk_gemm_bf16_nn": (
            [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_f, c_int, c_vp],
            c_int,
        ),
        "bk_gemm_bf16_nn_ok": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int], c_int),
        "bk_transpose_bf16": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "bk_transpose_to_bf16": ([c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "bk_transpose": ([c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "bk_gemm_fp": ([c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_i64, c_i64, c_i64, c_vp], c_int),
        "bk_gemm_f32x6_workspace_bytes": ([c_int, c_int, c_int], c_i64),
        "bk_gemm_f32x6": (
            [c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp],
            c_int,
        ),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                path = library_path()
                if not os.path.exists(path):
                    raise BeekernError(
                        f"beekern kernel library not found at {path}; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)"
                    )
                _preload_torch_runtime()
                handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                _declare(handle)
                _lib = handle
    return _lib


def is_loaded() -> bool:
    return _lib is not None


def check(rc: int, what: str = "beekern") -> None:
    if rc == 0:
        return
    detail = ""
    try:
        msg = lib().bk_last_error()
        detail = msg.decode(errors="replace") if msg else ""
    except Exception:
        pass
    text = f"{what}: {STATUS.get(rc, rc)}" + (f" ({detail})" if detail else "")
    if rc == 4:
        raise QuotaExceeded(text)
    if rc == 3:
        raise MemoryError(text)
    raise BeekernError(text)
