"""Does /proc/self/pagemap report PM_MMAP_EXCLUSIVE for the pages a forked
child copied?  (the zygote's copy-on-write prefault learns from it)"""
import ctypes
import mmap
import os
import struct

N = 64
buf = mmap.mmap(-1, N * 4096, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
for i in range(N):
    buf[i * 4096] = 1
addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
print("kernel", os.uname().release, "uid", os.getuid(), flush=True)
pid = os.fork()
if pid == 0:
    for i in range(0, N, 4):
        buf[i * 4096] = 2
    with open("/proc/self/pagemap", "rb") as f:
        f.seek(addr // 4096 * 8)
        ent = struct.unpack("%dQ" % N, f.read(N * 8))
    bits = "".join("X" if (e >> 56) & 1 else ("p" if e >> 63 else ".") for e in ent)
    print("child  ", bits, flush=True)
    os._exit(0)
os.waitpid(pid, 0)
