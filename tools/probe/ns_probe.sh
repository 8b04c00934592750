id; cat /proc/sys/user/max_user_namespaces; cat /proc/sys/kernel/unprivileged_userns_clone 2>/dev/null; cat /proc/sys/kernel/apparmor_restrict_unprivileged_userns 2>/dev/null
unshare -Um sh -c 'echo inns; id; mount -t tmpfs none /mnt && echo mounted_tmpfs; mount --rbind /dev /mnt && echo rbind_ok; ls /mnt | head -3'; echo unshare_rc=$?
python - <<'PY'
import os, ctypes
print("threads before torch", len(os.listdir("/proc/self/task")))
import numpy
print("threads after numpy", len(os.listdir("/proc/self/task")))
import torch
print("threads after torch", len(os.listdir("/proc/self/task")))
PY
