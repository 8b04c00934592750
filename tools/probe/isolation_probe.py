"""Probe which isolation primitives this kernel/container grants the current
user: Landlock ABI, seccomp filters, unprivileged user namespaces, a writable
cgroup v2 subtree, setuid capability, device node groups."""
import ctypes, json, os, subprocess, sys

libc = ctypes.CDLL(None, use_errno=True)
out = {"uid": os.getuid(), "euid": os.geteuid(), "groups": os.getgroups(), "kernel": os.uname().release}
# landlock_create_ruleset(NULL, 0, LANDLOCK_CREATE_RULESET_VERSION)
r = libc.syscall(444, None, ctypes.c_size_t(0), ctypes.c_uint32(1))
out["landlock_abi"] = r if r >= 0 else -ctypes.get_errno()
try:
    out["lsm"] = open("/sys/kernel/security/lsm").read().strip()
except OSError as e:
    out["lsm"] = str(e)
out["seccomp_actions"] = open("/proc/sys/kernel/seccomp/actions_avail").read().strip() if os.path.exists("/proc/sys/kernel/seccomp/actions_avail") else None
for k in ("/proc/sys/kernel/unprivileged_userns_clone", "/proc/sys/user/max_user_namespaces", "/proc/sys/kernel/pid_max", "/proc/sys/kernel/threads-max"):
    try:
        out[k] = open(k).read().strip()
    except OSError as e:
        out[k] = str(e)
p = subprocess.run(["unshare", "-U", "-r", "-p", "-f", "-m", "--mount-proc", "sh", "-c", "id; ls /proc | head -3"], capture_output=True, text=True)
out["userns_pidns_mountproc"] = [p.returncode, p.stdout.strip(), p.stderr.strip()[:200]]
p = subprocess.run(["unshare", "-U", "sh", "-c", "id"], capture_output=True, text=True)
out["userns"] = [p.returncode, p.stdout.strip(), p.stderr.strip()[:200]]
try:
    cg = open("/proc/self/cgroup").read().strip()
    out["cgroup"] = cg
    path = "/sys/fs/cgroup" + cg.split("::", 1)[1] if "::" in cg else None
    out["cgroup_path"] = path
    if path:
        out["cgroup_controllers"] = open(os.path.join(path, "cgroup.controllers")).read().strip() if os.path.exists(os.path.join(path, "cgroup.controllers")) else None
        out["cgroup_subtree_control"] = open(os.path.join(path, "cgroup.subtree_control")).read().strip() if os.path.exists(os.path.join(path, "cgroup.subtree_control")) else None
        out["cgroup_writable"] = os.access(path, os.W_OK)
        t = os.path.join(path, "bee-probe")
        try:
            os.mkdir(t); out["cgroup_mkdir"] = True; os.rmdir(t)
        except OSError as e:
            out["cgroup_mkdir"] = str(e)
except OSError as e:
    out["cgroup"] = str(e)
for dev in ("/dev/kfd", "/dev/dri"):
    try:
        st = os.stat(dev); out[dev] = [st.st_uid, st.st_gid, oct(st.st_mode)]
        if dev == "/dev/dri":
            out["dri_nodes"] = {n: [os.stat("/dev/dri/" + n).st_gid, oct(os.stat("/dev/dri/" + n).st_mode)] for n in os.listdir(dev)}
    except OSError as e:
        out[dev] = str(e)
print(json.dumps(out, indent=1))
