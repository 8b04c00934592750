"""Box probe: HIP init cost in forked workers (from a torch-imported zygote)."""
import ctypes, os, sys, time, json, subprocess
t0 = time.time()
import torch  # noqa
import numpy  # noqa
t_imp = time.time() - t0
print("import torch+numpy s", round(t_imp, 3), "cuda initialized:", torch.cuda.is_initialized(), flush=True)
here = os.path.dirname(os.path.abspath(__file__))

def child(tag, use_torch=False):
    r = {}
    t = time.time()
    if use_torch:
        x = torch.zeros(1, device="cuda"); torch.cuda.synchronize()
        r["torch_first_tensor_s"] = time.time() - t
        t = time.time(); y = torch.randn(1024, 1024, device="cuda"); z = y @ y; torch.cuda.synchronize()
        r["torch_first_matmul_s"] = time.time() - t
        free, total = torch.cuda.mem_get_info()
        r["free_gb"] = free / 1e9; r["total_gb"] = total / 1e9
        return r
    hip = ctypes.CDLL("libamdhip64.so.7")
    r["dlopen_s"] = time.time() - t; t = time.time()
    rc = hip.hipInit(0); r["hipInit_s"] = time.time() - t; r["hipInit_rc"] = rc; t = time.time()
    n = ctypes.c_int(); hip.hipGetDeviceCount(ctypes.byref(n)); r["ndev"] = n.value
    hip.hipSetDevice(0); rc = hip.hipFree(None); r["ctx_s"] = time.time() - t; r["ctx_rc"] = rc; t = time.time()
    free = ctypes.c_size_t(); total = ctypes.c_size_t(); hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
    r["free_gb"] = free.value / 1e9; r["total_gb"] = total.value / 1e9
    p = ctypes.c_void_p(); rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30)); r["malloc1g_s"] = time.time() - t; r["malloc_rc"] = rc; t = time.time()
    lib = ctypes.CDLL(os.path.join(here, "libprobe.so"))
    r["dlopen_lib_s"] = time.time() - t; t = time.time()
    rc = lib.probe_fill(p, ctypes.c_float(1.0), ctypes.c_long(1 << 28), None); hip.hipDeviceSynchronize()
    r["first_launch_s"] = time.time() - t; r["launch_rc"] = rc; t = time.time()
    for _ in range(100): lib.probe_fill(p, ctypes.c_float(2.0), ctypes.c_long(1 << 28), None)
    hip.hipDeviceSynchronize(); r["100_fills_1GB_s"] = time.time() - t
    return r

def run_forks(k, use_torch=False):
    t = time.time(); pids = []
    for i in range(k):
        rfd, wfd = os.pipe()
        pid = os.fork()
        if pid == 0:
            os.close(rfd)
            try:
                res = child(i, use_torch)
            except Exception as e:
                res = {"err": repr(e)}
            os.write(wfd, json.dumps(res).encode()); os._exit(0)
        os.close(wfd); pids.append((pid, rfd))
    outs = []
    for pid, rfd in pids:
        data = b""
        while True:
            b = os.read(rfd, 65536)
            if not b: break
            data += b
        os.waitpid(pid, 0); outs.append(json.loads(data))
    return time.time() - t, outs

for k in (1, 1, 4, 16):
    wall, outs = run_forks(k)
    print(f"hip forks k={k} wall={wall:.3f}", json.dumps(outs[0]), flush=True)
    if k > 1:
        print("  max hipInit+ctx", max(o.get("hipInit_s", 0) + o.get("ctx_s", 0) for o in outs), flush=True)
for k in (1, 4):
    wall, outs = run_forks(k, use_torch=True)
    print(f"torch forks k={k} wall={wall:.3f}", json.dumps(outs[0]), flush=True)
def sh(c):
    p = subprocess.run(c, shell=True, capture_output=True, text=True)
    return (p.returncode, p.stdout.strip()[-600:], p.stderr.strip()[-300:])
for c in ["whoami", "nproc", "df -h /dev/shm /tmp .", "ulimit -a | head -20", "unshare -Ur true", "unshare -Urm true", "unshare -Urn true", "unshare -Urp --fork true",
          "cat /proc/sys/kernel/unprivileged_userns_clone", "cat /proc/sys/user/max_user_namespaces", "rocm-smi --showmeminfo vram | head -20", "python -c 'import os;print(os.sched_getaffinity(0))'"]:
    print(c, "->", sh(c), flush=True)
