"""Out-of-process VRAM accounting for the executor's HBM watchdog: which
source shows a sandbox's device memory?  A child allocates 1 GiB with torch;
the parent reads (a) KFD sysfs /sys/class/kfd/kfd/proc/<pid> (host pids: may
not match in a pid namespace) and (b) DRM fdinfo of the child's render-node
descriptors (drm-memory-vram, per DRM client)."""
import json, os, subprocess, sys, time

child = subprocess.Popen([sys.executable, "-c",
    "import torch,sys,time; x=torch.empty(1<<30,dtype=torch.uint8,device='cuda'); torch.cuda.synchronize(); "
    "print('ready',flush=True); time.sleep(20)"], stdout=subprocess.PIPE, text=True)
out = {"child_ready": child.stdout.readline().strip(), "pid": child.pid}
fds = f"/proc/{child.pid}/fd"
for fd in sorted(os.listdir(fds), key=int):
    try:
        target = os.readlink(os.path.join(fds, fd))
    except OSError:
        continue
    if "dri" in target or "kfd" in target:
        try:
            info = open(f"/proc/{child.pid}/fdinfo/{fd}").read()
        except OSError as e:
            info = f"ERR {e}"
        out[f"fd{fd}:{target}"] = [l for l in info.splitlines() if l.startswith("drm-") or "vram" in l.lower()][:20]
try:
    out["kfd_proc_list"] = sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:20]
except OSError as e:
    out["kfd_proc_error"] = str(e)
child.kill()
print(json.dumps(out, indent=1))
