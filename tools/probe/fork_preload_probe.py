# fork+_exit CPU (parent and child) of a gc-frozen interpreter by preloaded modules:
# what a zygote's preload costs every sandbox forked from it.
# usage: python tools/probe/fork_preload_probe.py "numpy,bee_code_interpreter_fs_amd.ops"
import os, sys, time, resource, gc
mods = sys.argv[1].split(",") if sys.argv[1] else []
for m in mods: __import__(m)
gc.collect(); gc.freeze()
N=300
r0=resource.getrusage(resource.RUSAGE_SELF); c0=resource.getrusage(resource.RUSAGE_CHILDREN)
t=time.perf_counter()
for i in range(N):
    pid=os.fork()
    if pid==0:
        os._exit(0)
    os.waitpid(pid,0)
dt=time.perf_counter()-t
r1=resource.getrusage(resource.RUSAGE_SELF); c1=resource.getrusage(resource.RUSAGE_CHILDREN)
par=(r1.ru_utime+r1.ru_stime-r0.ru_utime-r0.ru_stime)/N*1e3
ch=(c1.ru_utime+c1.ru_stime-c0.ru_utime-c0.ru_stime)/N*1e3
rss=open('/proc/self/status').read().split('VmRSS:')[1].split()[0]
print(f"{sys.argv[1] or 'bare':40s} wall/fork {dt/N*1e3:.3f} ms parent cpu {par:.3f} child cpu {ch:.3f} rss {rss} kB")
