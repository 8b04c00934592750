"""Native build: HIP kernels (gfx950), the C++ executor daemon, the HBM-quota
interposer and the RCCL bench.  Incremental (mtime) and parallel.

Invoked by ``__graft_entry__.build()`` and ``python -m bee_code_interpreter_fs_amd._build``.
hipcc cross-compiles for gfx950 without a GPU present.
"""

from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass, field
from typing import List, Sequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bee_code_interpreter_fs_amd")
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("BEE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", os.path.join(ROCM, "bin", "hipcc"))
CXX = os.environ.get("CXX", "g++")

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-Wno-unused-value",
    "-Wno-unused-result",
]


@dataclass
class Target:
    name: str
    output: str
    sources: List[str]
    compiler: str
    compile_flags: List[str]
    link_flags: List[str] = field(default_factory=list)
    shared: bool = True
    headers: List[str] = field(default_factory=list)
    hip: bool = False
    optional: bool = False  # built only when named explicitly


def _targets() -> List[Target]:
    k = os.path.join(CSRC, "kernels")
    ex = os.path.join(CSRC, "executor")
    q = os.path.join(CSRC, "hbm_quota")
    # broker_fuzz.cpp / admission_test.cpp are CPU test harnesses' main()s,
    # not part of the daemon
    ex_srcs = sorted(os.path.join(ex, f) for f in os.listdir(ex)
                     if f.endswith(".cpp") and f not in ("broker_fuzz.cpp", "admission_test.cpp")) if os.path.isdir(ex) else []
    ex_hdrs = sorted(os.path.join(ex, f) for f in os.listdir(ex) if f.endswith(".hpp")) if os.path.isdir(ex) else []
    rb = os.path.join(CSRC, "rccl_bench")
    targets = [
        Target(
            name="beekern",
            output=os.path.join(PKG, "ops", "lib", "libbeekern.so"),
            sources=[os.path.join(k, f) for f in ("random.hip", "elementwise.hip", "reduce.hip", "gemm_bf16.hip", "gemm_bf16_256.hip", "gemm_bf16_256x.hip", "gemm_fp.hip", "runtime.cpp")],
            compiler=HIPCC,
            compile_flags=HIP_FLAGS,
            link_flags=[f"--offload-arch={ARCH}", "-shared", "-fPIC"],
            headers=[os.path.join(k, f) for f in ("bk_common.hpp", "bk_philox.hpp", "gemm256_impl.hpp", "gemm256w4_impl.hpp")],
            hip=True,
        ),
    ]
    if os.path.isdir(ex) and os.listdir(ex):
        targets.append(
            Target(
                name="bee-executor",
                output=os.path.join(PKG, "bin", "bee-executor"),
                sources=ex_srcs,
                compiler=CXX,
                compile_flags=[
                    "-O2", "-g", "-std=c++17", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Wno-unused-result",
                    "-pthread", f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__",
                ],
                link_flags=["-pthread", f"-L{ROCM}/lib", "-lamdhip64", "-lrocprofiler-sdk-roctx", "-ldl",
                            f"-Wl,-rpath,{ROCM}/lib"],
                shared=False,
                headers=sorted(os.path.join(ex, f) for f in os.listdir(ex) if f.endswith(".hpp")),
            )
        )
    if os.path.isdir(q) and os.listdir(q):
        targets.append(
            Target(
                name="hbm-quota",
                output=os.path.join(PKG, "lib", "libbee_hbm_quota.so"),
                sources=sorted(os.path.join(q, f) for f in os.listdir(q) if f.endswith(".cpp")),
                compiler=CXX,
                compile_flags=["-O2", "-fPIC", "-std=c++17", "-Wall", f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__"],
                link_flags=["-shared", "-fPIC", "-ldl", "-pthread"],
            )
        )
    # host sanitizer builds of the executor (opt-in: `python -m
    # bee_code_interpreter_fs_amd._build bee-executor-asan bee-executor-tsan`);
    # the daemon is host code only, so these are ordinary g++ sanitizers
    for san, flags in (("asan", ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-static-libasan"]),
                       ("tsan", ["-fsanitize=thread", "-fno-omit-frame-pointer"])):
        extra = ["-include", os.path.join(CSRC, "sanitize", "tsan_compat.hpp")] if san == "tsan" else []
        if ex_srcs:
            targets.append(
                Target(
                    name=f"bee-executor-{san}",
                    output=os.path.join(ROOT, "build", "sanitize", f"bee-executor-{san}"),
                    sources=ex_srcs,
                    compiler=CXX,
                    compile_flags=["-O1", "-g", "-std=c++17", "-pthread", f"-I{ROCM}/include",
                                   "-D__HIP_PLATFORM_AMD__", *flags, *extra],
                    link_flags=[*flags, "-pthread", f"-L{ROCM}/lib", "-lamdhip64", "-lrocprofiler-sdk-roctx", "-ldl",
                                f"-Wl,-rpath,{ROCM}/lib"],
                    shared=False,
                    headers=ex_hdrs,
                    optional=True,
                )
            )
    if ex_srcs:
        # the broker's protocol core over a host-memory device, under
        # ASan/UBSan: what tests/test_broker_fuzz_cpu.py drives with hostile frames
        targets.append(
            Target(
                name="broker-fuzz",
                output=os.path.join(ROOT, "build", "sanitize", "bee-broker-fuzz"),
                sources=[os.path.join(ex, "broker_core.cpp"), os.path.join(ex, "broker_fuzz.cpp")],
                compiler=CXX,
                compile_flags=["-O1", "-g", "-std=c++17", "-Wall", "-Wextra", "-fsanitize=address,undefined",
                               "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
                link_flags=["-fsanitize=address,undefined", "-static-libasan"],
                shared=False,
                headers=[os.path.join(ex, "broker_core.hpp")],
            )
        )
    if ex_srcs:
        # the admission state machine alone, under ThreadSanitizer: what
        # tests/test_admission_unit_cpu.py drives (no daemon, no service)
        targets.append(
            Target(
                name="admission-test",
                output=os.path.join(ROOT, "build", "sanitize", "bee-admission-test"),
                sources=[os.path.join(ex, "admission.cpp"), os.path.join(ex, "admission_test.cpp")],
                compiler=CXX,
                compile_flags=["-O1", "-g", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-fsanitize=thread",
                               "-fno-omit-frame-pointer", "-include", os.path.join(CSRC, "sanitize", "tsan_compat.hpp")],
                link_flags=["-fsanitize=thread", "-pthread"],
                shared=False,
                headers=[os.path.join(ex, "admission.hpp"), os.path.join(CSRC, "sanitize", "tsan_compat.hpp")],
            )
        )
    fm = os.path.join(CSRC, "fsmap")
    if os.path.isdir(fm) and os.listdir(fm):
        targets.append(
            Target(
                name="fsmap",
                output=os.path.join(PKG, "lib", "libbee_fsmap.so"),
                sources=sorted(os.path.join(fm, f) for f in os.listdir(fm) if f.endswith(".cpp")),
                compiler=CXX,
                compile_flags=["-O2", "-fPIC", "-std=c++17", "-Wall", "-U_FORTIFY_SOURCE", "-fvisibility=default"],
                link_flags=["-shared", "-fPIC", "-ldl"],
            )
        )
    lab = os.path.join(ROOT, "tools", "gemm_lab")
    if os.path.isdir(lab):
        targets.append(
            Target(
                name="gemm-lab",
                output=os.path.join(lab, "libgemmlab.so"),
                sources=[os.path.join(lab, "gemm_lab.hip")],
                compiler=HIPCC,
                # accumulators in the VGPR form of MFMA: the 4-wave kernel's
                # 256 accumulators + fragments otherwise bounce through AGPR moves
                compile_flags=HIP_FLAGS + ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
                link_flags=[f"--offload-arch={ARCH}", "-shared", "-fPIC"],
                headers=[os.path.join(k, "bk_common.hpp"), os.path.join(k, "gemm256_impl.hpp"), os.path.join(k, "gemm256w4_impl.hpp")],
                hip=True,
                optional=True,
            )
        )
    zl = os.path.join(CSRC, "zygote")
    if os.path.isdir(zl):
        import sysconfig

        targets.append(
            Target(
                name="zygote-loop",
                output=os.path.join(PKG, "runtime", "_zygote_loop" + sysconfig.get_config_var("EXT_SUFFIX")),
                sources=[os.path.join(zl, "zygote_loop.cpp")],
                compiler=CXX,
                compile_flags=["-O2", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-Wno-missing-field-initializers",
                               f"-I{sysconfig.get_paths()['include']}"],
                link_flags=["-shared", "-fPIC"],
            )
        )
    jl = os.path.join(CSRC, "jail")
    if os.path.isdir(jl):
        import sysconfig

        targets.append(
            Target(
                name="jail",
                output=os.path.join(PKG, "runtime", "_jail" + sysconfig.get_config_var("EXT_SUFFIX")),
                sources=[os.path.join(jl, "jail.cpp")],
                compiler=CXX,
                compile_flags=["-O2", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-Wno-missing-field-initializers",
                               f"-I{sysconfig.get_paths()['include']}"],
                link_flags=["-shared", "-fPIC"],
            )
        )
    if os.path.isdir(rb) and os.listdir(rb):
        targets.append(
            Target(
                name="rccl-bench",
                output=os.path.join(PKG, "bin", "bee-rccl-bench"),
                sources=sorted(os.path.join(rb, f) for f in os.listdir(rb) if f.endswith(".cpp")),
                compiler=HIPCC,
                compile_flags=HIP_FLAGS + [f"-I{ROCM}/include"],
                link_flags=[f"--offload-arch={ARCH}", f"-L{ROCM}/lib", "-lrccl", "-pthread"],
                shared=False,
                hip=True,
            )
        )
    return targets


def _stale(output: str, inputs: Sequence[str]) -> bool:
    if not os.path.exists(output):
        return True
    out_m = os.path.getmtime(output)
    return any(os.path.getmtime(i) > out_m for i in inputs if os.path.exists(i))


def _run(cmd: List[str]) -> None:
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")


def _compile(t: Target, src: str) -> str:
    os.makedirs(OBJ, exist_ok=True)
    obj = os.path.join(OBJ, f"{t.name}__{os.path.basename(src)}.o")
    if _stale(obj, [src, *t.headers, __file__]):
        extra = ["-x", "hip"] if (t.hip and src.endswith(".cpp")) else []
        _run([t.compiler, *t.compile_flags, *extra, "-c", src, "-o", obj])
    return obj


def build(targets: Sequence[str] = (), jobs: int = 0, verbose: bool = True) -> List[str]:
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    every = _targets()
    chosen = [t for t in every if t.name in targets] if targets else [t for t in every if not t.optional]
    jobs = jobs or min(8, os.cpu_count() or 4)
    built = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as pool:
        futures = {t.name: [pool.submit(_compile, t, s) for s in t.sources] for t in chosen}
        for t in chosen:
            objs = [f.result() for f in futures[t.name]]
            if _stale(t.output, objs):
                os.makedirs(os.path.dirname(t.output), exist_ok=True)
                tmp = t.output + ".tmp"
                _run([t.compiler, *objs, *t.link_flags, "-o", tmp])
                os.replace(tmp, t.output)
                if verbose:
                    print(f"[build] {t.name} -> {os.path.relpath(t.output, ROOT)}", flush=True)
            built.append(t.output)
    return built


if __name__ == "__main__":
    build(sys.argv[1:])
