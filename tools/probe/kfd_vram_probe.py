"""Does the KFD sysfs expose per-process VRAM use (the HBM watchdog's
out-of-process source)?  A child allocates 1 GiB with torch; the parent
lists /sys/class/kfd/kfd/proc/<child>/ and reads every vram_* file."""
import json, os, subprocess, sys, time

child = subprocess.Popen([sys.executable, "-c",
    "import torch,sys,time; x=torch.empty(1<<30,dtype=torch.uint8,device='cuda'); torch.cuda.synchronize(); "
    "print('ready',flush=True); time.sleep(20)"], stdout=subprocess.PIPE, text=True)
line = child.stdout.readline().strip()
out = {"child_ready": line}
base = f"/sys/class/kfd/kfd/proc/{child.pid}"
try:
    out["entries"] = sorted(os.listdir(base))
    for e in out["entries"]:
        p = os.path.join(base, e)
        if os.path.isfile(p):
            try:
                out[e] = open(p).read().strip()[:200]
            except OSError as ex:
                out[e] = f"ERR {ex}"
        elif os.path.isdir(p):
            out[e + "/"] = sorted(os.listdir(p))[:20]
except OSError as e:
    out["error"] = str(e)
try:
    out["kfd_proc_list"] = sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:50]
    out["topology_nodes"] = sorted(os.listdir("/sys/class/kfd/kfd/topology/nodes"))
    for n in out["topology_nodes"]:
        p = f"/sys/class/kfd/kfd/topology/nodes/{n}/gpu_id"
        out[f"node{n}_gpu_id"] = open(p).read().strip()
except OSError as e:
    out["error2"] = str(e)
child.kill()
print(json.dumps(out, indent=1))
