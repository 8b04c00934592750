// Sandbox jail: the isolation boundary applied to every single-use sandbox
// process right after it is forked from its zygote, before any user code
// runs.  Python extension `_jail` (bee_code_interpreter_fs_amd/runtime).
//
// The reference isolates each execution in a fresh Kubernetes pod running as
// a non-root UID (`src/code_interpreter/services/kubernetes_code_executor.py:
// 220-253`, `executor/Dockerfile:91-98`): the pod cannot see the service's
// file-object store, other pods, or the service's processes.  Forked
// sandboxes share one host, so the same guarantees are rebuilt from kernel
// primitives, each applied when the kernel/privileges allow it:
//
//   * a per-sandbox UID/GID (service running with CAP_SETUID): DAC keeps the
//     sandbox out of the store (0700), other sandboxes' dirs (0700, other
//     UIDs), the control sockets (0600) and other processes (signals,
//     /proc/<pid>/environ);  RLIMIT_NPROC becomes a per-sandbox pids cap;
//   * Landlock (unprivileged, ABI >= 1): default-deny filesystem view --
//     read/execute on the system and Python trees, read-write only on the
//     sandbox's own workspace/runtime-packages/tmp and /dev/shm; protected
//     trees (store, sandbox root, control dir) are carved out of every
//     allowed hierarchy.  Landlock also scopes ptrace (so /proc/<pid>/environ,
//     /mem, /fd of processes outside the sandbox are denied), and from ABI 6
//     signals and abstract Unix sockets to the sandbox's own domain;
//   * seccomp-bpf: kernel-attack-surface syscalls (ptrace, process_vm_*,
//     mount/namespace/bpf/perf/keyring/module/kexec/io_uring ...) and clone
//     with namespace flags fail with EPERM, clone3 with ENOSYS (libc falls
//     back to clone); non-native syscall ABIs (x32, i386) kill the process;
//   * rlimits: no core dumps, a per-process data-segment cap (RLIMIT_DATA:
//     private writable memory -- a 100 GB bytearray is a MemoryError), file
//     size cap, and the pids cap above.
//
// prepare() runs once in the zygote: it resolves the static rule set and
// opens one O_PATH descriptor per rule, so a sandbox pays only one
// landlock_add_rule per rule (no path walks) when it applies the jail.
#include <Python.h>

#include <errno.h>
#include <fcntl.h>
#include <grp.h>
#include <linux/audit.h>
#include <linux/capability.h>
#include <linux/filter.h>
#include <linux/landlock.h>
#include <linux/seccomp.h>
#include <stddef.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstring>
#include <string>
#include <vector>

namespace {

// ---- Landlock --------------------------------------------------------------------

// access rights, by ABI version that introduced them
constexpr uint64_t kFsV1 = (1ULL << 13) - 1;          // EXECUTE .. MAKE_SYM
constexpr uint64_t kFsRefer = 1ULL << 13;             // ABI 2
constexpr uint64_t kFsTruncate = 1ULL << 14;          // ABI 3
constexpr uint64_t kScopeAbstractUnix = 1ULL << 0;    // ABI 6
constexpr uint64_t kScopeSignal = 1ULL << 1;          // ABI 6

constexpr uint64_t kRead = LANDLOCK_ACCESS_FS_EXECUTE | LANDLOCK_ACCESS_FS_READ_FILE | LANDLOCK_ACCESS_FS_READ_DIR;

// ruleset_attr grew over ABI versions; pass the size the kernel knows
struct RulesetAttr {
  uint64_t handled_access_fs;
  uint64_t handled_access_net;
  uint64_t scoped;
};

int ll_abi() {
  static int abi = -2;
  if (abi == -2) {
    const long r = syscall(__NR_landlock_create_ruleset, nullptr, 0, LANDLOCK_CREATE_RULESET_VERSION);
    abi = r < 0 ? 0 : (int)r;
  }
  return abi;
}

uint64_t handled_fs(int abi) {
  uint64_t m = kFsV1;
  if (abi >= 2) m |= kFsRefer;
  if (abi >= 3) m |= kFsTruncate;
  // IOCTL_DEV (ABI 5) is deliberately not handled: HIP drives /dev/kfd and
  // the render node with ioctls, and device access is already mediated by
  // the device nodes' own permissions
  return m;
}

struct Rule {
  int fd;
  uint64_t access;  // requested; masked by handled_fs() at apply time
  std::string path;
};

std::vector<Rule> g_rules;  // static rules prepared in the zygote
constexpr int kRuleFdBase = 700;

// ---- seccomp ---------------------------------------------------------------------

// syscalls a sandbox never needs; they fail with EPERM
const int kDenied[] = {
    SYS_ptrace, SYS_process_vm_readv, SYS_process_vm_writev, SYS_kcmp, SYS_pidfd_getfd, SYS_process_madvise,
    SYS_mount, SYS_umount2, SYS_pivot_root, SYS_chroot, SYS_unshare, SYS_setns, SYS_fsopen, SYS_fsconfig,
    SYS_fsmount, SYS_fspick, SYS_move_mount, SYS_open_tree, SYS_mount_setattr, SYS_bpf, SYS_perf_event_open,
    SYS_userfaultfd, SYS_keyctl, SYS_add_key, SYS_request_key, SYS_init_module, SYS_finit_module,
    SYS_delete_module, SYS_kexec_load, SYS_kexec_file_load, SYS_reboot, SYS_swapon, SYS_swapoff, SYS_acct,
    SYS_quotactl, SYS_syslog, SYS_settimeofday, SYS_clock_settime, SYS_clock_adjtime, SYS_adjtimex,
    SYS_sethostname, SYS_setdomainname, SYS_iopl, SYS_ioperm, SYS_open_by_handle_at, SYS_name_to_handle_at,
    SYS_fanotify_init, SYS_lookup_dcookie, SYS_vhangup, SYS_io_uring_setup, SYS_io_uring_enter,
    SYS_io_uring_register, SYS_uselib, SYS_personality,
};

// clone(2) flags that create namespaces: refused (a sandbox never needs
// them, and on hosts that allow unprivileged user namespaces they reopen
// everything unshare/setns are denied for)
constexpr uint32_t kCloneNsMask = 0x00020000u /*NEWNS*/ | 0x02000000u /*NEWCGROUP*/ | 0x04000000u /*NEWUTS*/ |
                                  0x08000000u /*NEWIPC*/ | 0x10000000u /*NEWUSER*/ | 0x20000000u /*NEWPID*/ |
                                  0x40000000u /*NEWNET*/ | 0x00000080u /*NEWTIME*/;
constexpr uint32_t kPrSetChildSubreaper = 36;

// The program, in order:
//   arch != x86_64                          -> KILL_PROCESS (i386 ABI)
//   nr >= 0x40000000 (x32 aliases)          -> KILL_PROCESS
//   clone with a CLONE_NEW* flag            -> EPERM
//   clone3                                  -> ENOSYS (libc falls back to clone, whose flags are visible here;
//                                              clone3 passes them in memory the filter cannot read)
//   prctl(PR_SET_CHILD_SUBREAPER, 0)        -> EPERM (a sandbox leader is its tree's subreaper: orphans of its
//                                              processes stay under it, where the executor accounts and kills
//                                              them; it may not drop that)
//   any syscall of kDenied                  -> EPERM
//   everything else                         -> ALLOW
std::vector<sock_filter> seccomp_program() {
  std::vector<sock_filter> p;
  // forward jumps by label: (instruction index, which field, label)
  struct Fix {
    size_t at;
    bool jt;
    int label;
  };
  std::vector<Fix> fixes;
  enum { kAllow, kEperm, kKill, kEnosys, kClone, kPrctl, kAllowEnd, kEpermEnd, kLabels };
  size_t where[kLabels] = {};
  auto stmt = [&](uint16_t code, uint32_t k) { p.push_back(BPF_STMT(code, k)); };
  // conditional jump: true -> label jt (or fall through when < 0), false -> label jf (or fall through)
  auto jump = [&](uint16_t code, uint32_t k, int jt, int jf) {
    if (jt >= 0) fixes.push_back({p.size(), true, jt});
    if (jf >= 0) fixes.push_back({p.size(), false, jf});
    p.push_back(BPF_JUMP(code, k, 0, 0));
  };
  auto label = [&](int l) { where[l] = p.size(); };
  auto arg_lo = [](int i) { return (uint32_t)(offsetof(seccomp_data, args) + 8 * i); };
  auto arg_hi = [](int i) { return (uint32_t)(offsetof(seccomp_data, args) + 8 * i + 4); };

  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(seccomp_data, arch));
  jump(BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, -1, kKill);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(seccomp_data, nr));
  jump(BPF_JMP | BPF_JGE | BPF_K, 0x40000000u, kKill, -1);
  jump(BPF_JMP | BPF_JEQ | BPF_K, SYS_clone, kClone, -1);
  jump(BPF_JMP | BPF_JEQ | BPF_K, SYS_clone3, kEnosys, -1);
  jump(BPF_JMP | BPF_JEQ | BPF_K, SYS_prctl, kPrctl, -1);
  for (int nr : kDenied) jump(BPF_JMP | BPF_JEQ | BPF_K, (uint32_t)nr, kEperm, -1);
  label(kAllow);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ALLOW);
  label(kEperm);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA));
  label(kKill);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS);
  label(kEnosys);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (ENOSYS & SECCOMP_RET_DATA));
  label(kClone);  // the kernel takes the low 32 bits of clone's flags
  stmt(BPF_LD | BPF_W | BPF_ABS, arg_lo(0));
  jump(BPF_JMP | BPF_JSET | BPF_K, kCloneNsMask, kEpermEnd, kAllowEnd);
  label(kPrctl);  // option is an int (low 32 bits); arg2 is the full unsigned long
  stmt(BPF_LD | BPF_W | BPF_ABS, arg_lo(0));
  jump(BPF_JMP | BPF_JEQ | BPF_K, kPrSetChildSubreaper, -1, kAllowEnd);
  stmt(BPF_LD | BPF_W | BPF_ABS, arg_lo(1));
  jump(BPF_JMP | BPF_JEQ | BPF_K, 0, -1, kAllowEnd);
  stmt(BPF_LD | BPF_W | BPF_ABS, arg_hi(1));
  jump(BPF_JMP | BPF_JEQ | BPF_K, 0, kEpermEnd, kAllowEnd);
  // (BPF jumps only forward: the argument checks end in returns of their own)
  label(kAllowEnd);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ALLOW);
  label(kEpermEnd);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA));
  for (auto& f : fixes) {
    if (where[f.label] <= f.at || where[f.label] - f.at - 1 > 255) abort();  // forward, in range
    const size_t off = where[f.label] - f.at - 1;
    if (f.jt) p[f.at].jt = (uint8_t)off;
    else p[f.at].jf = (uint8_t)off;
  }
  return p;
}

bool seccomp_available() {
  // PR_GET_SECCOMP works everywhere seccomp is compiled in
  return prctl(PR_GET_SECCOMP, 0, 0, 0, 0) >= 0;
}

bool install_filter() {
  static std::vector<sock_filter> prog = seccomp_program();
  sock_fprog fp{(unsigned short)prog.size(), prog.data()};
  return syscall(SYS_seccomp, SECCOMP_SET_MODE_FILTER, 0, &fp) == 0;
}

// ---- helpers ---------------------------------------------------------------------

bool list_of_str(PyObject* o, std::vector<std::string>* out) {
  if (o == nullptr || o == Py_None) return true;
  PyObject* seq = PySequence_Fast(o, "expected a sequence of str");
  if (!seq) return false;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = PySequence_Fast_GET_ITEM(seq, i);
    const char* s = PyUnicode_AsUTF8(it);
    if (!s) {
      Py_DECREF(seq);
      return false;
    }
    out->push_back(s);
  }
  Py_DECREF(seq);
  return true;
}

long long dict_int(PyObject* d, const char* key, long long dflt) {
  PyObject* v = PyDict_GetItemString(d, key);  // borrowed
  if (!v || v == Py_None) return dflt;
  const long long r = PyLong_AsLongLong(v);
  if (r == -1 && PyErr_Occurred()) {
    PyErr_Clear();
    return dflt;
  }
  return r;
}

bool dict_bool(PyObject* d, const char* key, bool dflt) {
  PyObject* v = PyDict_GetItemString(d, key);
  if (!v || v == Py_None) return dflt;
  return PyObject_IsTrue(v) == 1;
}

PyObject* os_error(const char* what) {
  const int e = errno;
  PyErr_Format(PyExc_OSError, "jail: %s: %s", what, strerror(e));
  return nullptr;
}

bool set_limit(int res, long long v) {
  if (v <= 0) return true;
  rlimit rl{(rlim_t)v, (rlim_t)v};
  rlimit cur{};
  if (getrlimit(res, &cur) == 0 && cur.rlim_max != RLIM_INFINITY && (rlim_t)v > cur.rlim_max) rl.rlim_max = rl.rlim_cur = cur.rlim_max;
  return setrlimit(res, &rl) == 0;
}

// ---- Python API ------------------------------------------------------------------

PyObject* py_probe(PyObject*, PyObject*) {
  const int abi = ll_abi();
  const bool root = geteuid() == 0;
  return Py_BuildValue("{s:i,s:O,s:O,s:i,s:i}", "landlock_abi", abi, "seccomp", seccomp_available() ? Py_True : Py_False,
                       "can_setuid", root ? Py_True : Py_False, "euid", (int)geteuid(), "prepared_rules",
                       (int)g_rules.size());
}

// prepare([(path, access_mask), ...]) in the zygote: open the static rule set
PyObject* py_prepare(PyObject*, PyObject* args) {
  PyObject* rules;
  if (!PyArg_ParseTuple(args, "O", &rules)) return nullptr;
  for (auto& r : g_rules) close(r.fd);
  g_rules.clear();
  PyObject* seq = PySequence_Fast(rules, "expected a sequence of (path, access)");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  int next_fd = kRuleFdBase;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const char* path;
    unsigned long long access;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(seq, i), "sK", &path, &access)) {
      Py_DECREF(seq);
      return nullptr;
    }
    const int fd = open(path, O_PATH | O_CLOEXEC);
    if (fd < 0) continue;  // vanished / unreadable: simply not allowed
    // park the descriptors in one contiguous block so a sandbox closes them
    // with a single close_range after applying the rules
    const int hi = fcntl(fd, F_DUPFD_CLOEXEC, next_fd);
    close(fd);
    if (hi < 0) continue;
    next_fd = hi + 1;
    g_rules.push_back(Rule{hi, (uint64_t)access, path});
  }
  Py_DECREF(seq);
  return PyLong_FromSsize_t((Py_ssize_t)g_rules.size());
}

// apply(opts) in a freshly forked sandbox.  opts keys:
//   uid, gid (0/absent: keep), groups [gid...], own_rw [paths], extra_ro [paths],
//   nproc, data_bytes, fsize_bytes, nofile, landlock (bool), seccomp (bool),
//   scope_signal (bool), scope_abstract_unix (bool)
// Returns a dict describing what was applied; raises OSError when a requested
// privilege drop fails (fail closed).
PyObject* py_apply(PyObject*, PyObject* args) {
  PyObject* opts;
  if (!PyArg_ParseTuple(args, "O!", &PyDict_Type, &opts)) return nullptr;
  std::vector<std::string> own_rw, extra_ro, groups_s;
  if (!list_of_str(PyDict_GetItemString(opts, "own_rw"), &own_rw)) return nullptr;
  if (!list_of_str(PyDict_GetItemString(opts, "extra_ro"), &extra_ro)) return nullptr;
  std::vector<gid_t> groups;
  if (PyObject* g = PyDict_GetItemString(opts, "groups")) {
    PyObject* seq = PySequence_Fast(g, "groups must be a sequence");
    if (!seq) return nullptr;
    for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i)
      groups.push_back((gid_t)PyLong_AsLong(PySequence_Fast_GET_ITEM(seq, i)));
    Py_DECREF(seq);
  }
  const long long uid = dict_int(opts, "uid", 0), gid = dict_int(opts, "gid", uid);
  const bool want_ll = dict_bool(opts, "landlock", true), want_sc = dict_bool(opts, "seccomp", true);
  const bool scope_signal = dict_bool(opts, "scope_signal", true);
  const bool scope_abstract = dict_bool(opts, "scope_abstract_unix", true);
  // net_connect_ports (a list, possibly empty): TCP connect() only to these
  // ports, in the sandbox's own Landlock layer (a handful of rules: no cost
  // next to the filesystem rules -- unlike a deny-list layer on the zygote,
  // ~65k allow rules that every sandbox layer nested below it copies, +13 ms
  // per sandbox).  Absent: TCP left alone.  bind()/listen() are not handled.
  std::vector<long> connect_ports;
  bool net_handled = false;
  if (PyObject* np = PyDict_GetItemString(opts, "net_connect_ports")) {
    if (np != Py_None) {
      PyObject* seq = PySequence_Fast(np, "net_connect_ports must be a sequence of ints");
      if (!seq) return nullptr;
      for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i) {
        const long port = PyLong_AsLong(PySequence_Fast_GET_ITEM(seq, i));
        if (port == -1 && PyErr_Occurred()) {
          Py_DECREF(seq);
          return nullptr;
        }
        if (port >= 0 && port < 65536) connect_ports.push_back(port);
      }
      Py_DECREF(seq);
      net_handled = true;
    }
  }

  // 1. resource limits (lowering limits needs no privilege)
  {
    rlimit z{0, 0};
    setrlimit(RLIMIT_CORE, &z);
  }
  if (!set_limit(RLIMIT_DATA, dict_int(opts, "data_bytes", 0))) return os_error("RLIMIT_DATA");
  if (!set_limit(RLIMIT_FSIZE, dict_int(opts, "fsize_bytes", 0))) return os_error("RLIMIT_FSIZE");
  if (!set_limit(RLIMIT_NOFILE, dict_int(opts, "nofile", 0))) return os_error("RLIMIT_NOFILE");

  // the sandbox's own trees are opened while the process still has the
  // daemon's identity (a sandbox UID may not be able to walk to them by path)
  std::vector<int> own_fds, ro_fds;
  for (auto& p : own_rw) {
    const int fd = open(p.c_str(), O_PATH | O_CLOEXEC);
    if (fd >= 0) own_fds.push_back(fd);
  }
  for (auto& p : extra_ro) {
    const int fd = open(p.c_str(), O_PATH | O_CLOEXEC);
    if (fd >= 0) ro_fds.push_back(fd);
  }
  struct Closer {
    std::vector<int>& a;
    std::vector<int>& b;
    ~Closer() {
      for (int fd : a) close(fd);
      for (int fd : b) close(fd);
    }
  } closer{own_fds, ro_fds};

  // 2. identity: a UID/GID of the sandbox's own (needs CAP_SETUID/CAP_SETGID)
  if (uid > 0) {
    if (setgroups(groups.size(), groups.empty() ? nullptr : groups.data()) != 0) return os_error("setgroups");
    if (setresgid((gid_t)gid, (gid_t)gid, (gid_t)gid) != 0) return os_error("setresgid");
    // the pids cap is per real UID: set it before switching so it binds
    if (!set_limit(RLIMIT_NPROC, dict_int(opts, "nproc", 0))) return os_error("RLIMIT_NPROC");
    if (setresuid((uid_t)uid, (uid_t)uid, (uid_t)uid) != 0) return os_error("setresuid");
    if (getuid() != (uid_t)uid || geteuid() != (uid_t)uid) {
      errno = EPERM;
      return os_error("uid did not change");
    }
  }
  // Dumpability.  With a UID of its own, DAC already keeps everyone else out
  // of the sandbox's /proc entries (the UID switch cleared the flag: set it
  // back so the sandbox reads its own /proc/self normally).  Sharing the
  // daemon's UID as root: non-dumpable, so capability-less root siblings
  // cannot read each other's environment or memory.
  //
  // Only a sandbox that is still root stays non-dumpable: for any other UID
  // the kernel would then hand /proc/self/{environ,fd,mem} to root and lock
  // the sandbox out of its own entries.  Siblings sharing an unprivileged
  // UID can read each other's environ/maps (PTRACE_MODE_READ), never memory,
  // fds or cwd (Landlock's ptrace scope); the service, daemon and zygote are
  // non-dumpable themselves.
  prctl(PR_SET_DUMPABLE, (uid > 0 || geteuid() != 0) ? 1 : 0, 0, 0, 0);
  // both Landlock and unprivileged seccomp require it; also no setuid
  // binary or file capability can hand privileges back
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) return os_error("PR_SET_NO_NEW_PRIVS");

  // 3. Landlock
  int abi = want_ll ? ll_abi() : 0;
  int nrules = 0;
  uint64_t scoped = 0;
  constexpr uint64_t kNetConnectTcp = 1ULL << 1;  // LANDLOCK_ACCESS_NET_CONNECT_TCP (ABI 4)
  const bool net_layer = net_handled && abi >= 4;
  if (abi > 0) {
    const uint64_t fs = handled_fs(abi);
    RulesetAttr attr{fs, net_layer ? kNetConnectTcp : 0, 0};
    if (abi >= 6) {
      if (scope_signal) scoped |= kScopeSignal;
      if (scope_abstract) scoped |= kScopeAbstractUnix;
      attr.scoped = scoped;
    }
    const size_t attr_size = abi >= 6 ? sizeof(RulesetAttr) : abi >= 4 ? 16 : 8;
    const int rs = (int)syscall(__NR_landlock_create_ruleset, &attr, attr_size, 0);
    if (rs < 0) return os_error("landlock_create_ruleset");
    auto add = [&](int fd, uint64_t access) -> bool {
      landlock_path_beneath_attr pb{};
      pb.allowed_access = access & fs;
      pb.parent_fd = fd;
      if (pb.allowed_access == 0) return true;
      if (syscall(__NR_landlock_add_rule, rs, LANDLOCK_RULE_PATH_BENEATH, &pb, 0) != 0) {
        // a rule on a non-directory may only carry file rights
        pb.allowed_access &= LANDLOCK_ACCESS_FS_EXECUTE | LANDLOCK_ACCESS_FS_WRITE_FILE | LANDLOCK_ACCESS_FS_READ_FILE |
                             kFsTruncate;
        if (pb.allowed_access == 0 || syscall(__NR_landlock_add_rule, rs, LANDLOCK_RULE_PATH_BENEATH, &pb, 0) != 0)
          return false;
      }
      ++nrules;
      return true;
    };
    for (auto& r : g_rules) add(r.fd, r.access);
    for (int fd : own_fds) add(fd, fs);
    for (int fd : ro_fds) add(fd, kRead);
    if (net_layer) {
      struct {
        uint64_t allowed_access;
        uint64_t port;
      } __attribute__((packed)) rule{kNetConnectTcp, 0};
      for (long port : connect_ports) {
        rule.port = (uint64_t)port;
        if (syscall(__NR_landlock_add_rule, rs, 2 /*LANDLOCK_RULE_NET_PORT*/, &rule, 0) != 0) {
          close(rs);
          return os_error("landlock_add_rule (connect port)");
        }
        ++nrules;
      }
    }
    if (syscall(__NR_landlock_restrict_self, rs, 0) != 0) {
      close(rs);
      return os_error("landlock_restrict_self");
    }
    close(rs);
  }
  if (!g_rules.empty()) {
    // the rule descriptors are the zygote's: not the sandbox's business
    const int lo = g_rules.front().fd, hi = g_rules.back().fd;
    if (syscall(SYS_close_range, (unsigned)lo, (unsigned)hi, 0) != 0)
      for (auto& r : g_rules) close(r.fd);
    g_rules.clear();
  }

  if (geteuid() == 0) {
    // still root (no sandbox UID: layout not walkable by other UIDs, or UID
    // mode off): shed every capability, so DAC, dumpability and Landlock bind
    // this process like any unprivileged one.  Under Landlock, CAP_DAC_READ_
    // SEARCH stays: the view (not DAC) decides what is readable, and root-owned
    // trees below another user's 0700 $HOME (this package, LD_PRELOAD shims
    // that exec'd children must load) stay reachable.  It cannot read another
    // process's /proc entries (that takes CAP_SYS_PTRACE), and
    // open_by_handle_at is refused by the seccomp filter below.
    const uint64_t keep = abi > 0 ? (1ULL << CAP_DAC_READ_SEARCH) : 0;
    for (int c = 0; c <= CAP_LAST_CAP; ++c)
      if (!((keep >> c) & 1)) prctl(PR_CAPBSET_DROP, c, 0, 0, 0);
    prctl(PR_CAP_AMBIENT, PR_CAP_AMBIENT_CLEAR_ALL, 0, 0, 0);
    __user_cap_header_struct hdr{_LINUX_CAPABILITY_VERSION_3, 0};
    __user_cap_data_struct data[2] = {};
    data[0].effective = data[0].permitted = (uint32_t)keep;
    if (syscall(SYS_capset, &hdr, data) != 0) return os_error("capset");
  }

  // 4. seccomp (normally inherited: the zygote installed it before forking)
  bool sc = prctl(PR_GET_SECCOMP, 0, 0, 0, 0) == 2;
  if (want_sc && !sc && seccomp_available()) {
    if (!install_filter()) return os_error("seccomp");
    sc = true;
  }
  return Py_BuildValue("{s:i,s:i,s:i,s:K,s:O,s:i,s:O}", "uid", (int)getuid(), "gid", (int)getgid(), "landlock_abi",
                       abi, "scoped", (unsigned long long)scoped, "seccomp", sc ? Py_True : Py_False, "landlock_rules",
                       nrules, "net_connect_restricted", net_layer ? Py_True : Py_False);
}

// seal_zygote(): the syscall filter on the zygote itself, so every fork
// inherits it -- the kernel compiles a filter per installation (~0.25 ms),
// which each sandbox would otherwise pay.  The zygote needs none of the
// refused calls either.
PyObject* py_seal_zygote(PyObject*, PyObject*) {
  if (!seccomp_available()) Py_RETURN_FALSE;
  if (prctl(PR_GET_SECCOMP, 0, 0, 0, 0) == 2) Py_RETURN_TRUE;
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) return os_error("PR_SET_NO_NEW_PRIVS");
  if (!install_filter()) return os_error("seccomp");
  Py_RETURN_TRUE;
}

// seal_zygote_net(deny_ports) -> dict: a Landlock network layer on the
// zygote itself (ABI >= 4), inherited by every sandbox it forks: TCP bind and
// connect are allowed on every port except `deny_ports` (the service's own
// listeners).  Landlock network rules are allow-lists of single ports, so the
// layer holds one rule per allowed port -- built once here (~65k
// landlock_add_rule calls, ~65 ms).  Costly all the same: a sandbox's own
// filesystem layer is a nested domain, and nesting copies the parent's rules
// (+13 ms of CPU per sandbox measured), hence opt-in (APP_SANDBOX_NET_LAYER).
// Egress stays open, as in the reference's pods (examples/tcp.py).  Returns what was applied, or
// {"applied": False, "reason": ...} on kernels without Landlock networking.
PyObject* py_seal_zygote_net(PyObject*, PyObject* args) {
  PyObject* ports;
  if (!PyArg_ParseTuple(args, "O", &ports)) return nullptr;
  std::vector<bool> deny(65536, false);
  PyObject* seq = PySequence_Fast(ports, "deny_ports must be a sequence of ints");
  if (!seq) return nullptr;
  int ndeny = 0;
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i) {
    const long p = PyLong_AsLong(PySequence_Fast_GET_ITEM(seq, i));
    if (p == -1 && PyErr_Occurred()) {
      Py_DECREF(seq);
      return nullptr;
    }
    if (p > 0 && p < 65536 && !deny[p]) {
      deny[p] = true;
      ++ndeny;
    }
  }
  Py_DECREF(seq);
  const int abi = ll_abi();
  if (abi < 4)
    return Py_BuildValue("{s:O,s:i,s:s}", "applied", Py_False, "landlock_abi", abi, "reason",
                         "Landlock network rules need ABI >= 4");
  constexpr uint64_t kNetBind = 1ULL << 0, kNetConnect = 1ULL << 1;  // LANDLOCK_ACCESS_NET_{BIND,CONNECT}_TCP
  RulesetAttr attr{0, kNetBind | kNetConnect, 0};
  const int rs = (int)syscall(__NR_landlock_create_ruleset, &attr, (size_t)16, 0);
  if (rs < 0) return os_error("landlock_create_ruleset (net)");
  struct {
    uint64_t allowed_access;
    uint64_t port;
  } __attribute__((packed)) rule{};
  constexpr int kRuleNetPort = 2;  // LANDLOCK_RULE_NET_PORT
  rule.allowed_access = kNetBind | kNetConnect;
  for (int p = 0; p < 65536; ++p) {  // port 0: bind to an ephemeral port
    if (deny[p]) continue;
    rule.port = (uint64_t)p;
    if (syscall(__NR_landlock_add_rule, rs, kRuleNetPort, &rule, 0) != 0) {
      close(rs);
      return os_error("landlock_add_rule (net)");
    }
  }
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0 || syscall(__NR_landlock_restrict_self, rs, 0) != 0) {
    close(rs);
    return os_error("landlock_restrict_self (net)");
  }
  close(rs);
  return Py_BuildValue("{s:O,s:i,s:i}", "applied", Py_True, "landlock_abi", abi, "denied_ports", ndeny);
}

// listen_guard() -> int: one more seccomp filter on the calling sandbox (all
// its threads), whose accept / accept4 calls go to the executor daemon
// (SECCOMP_RET_USER_NOTIF) -- it accepts on the sandbox's behalf and hands
// over only connections from the sandbox's own process tree
// (csrc/executor/listen_guard.hpp).  Also refuses seccomp(2) filters that ask
// for a listener of their own: a later filter of the sandbox cannot take the
// notifications over.  Returns the listener descriptor (close-on-exec), for
// the daemon.
PyObject* py_listen_guard(PyObject*, PyObject*) {
  std::vector<sock_filter> p = {
      BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(seccomp_data, nr)),
      BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, SYS_accept, 3, 0),   // -> notify
      BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, SYS_accept4, 2, 0),  // -> notify
      BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, SYS_seccomp, 2, 0),  // -> flags check
      BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW),
      BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_USER_NOTIF),
      BPF_STMT(BPF_LD | BPF_W | BPF_ABS, (uint32_t)(offsetof(seccomp_data, args) + 8)),  // flags (low word)
      BPF_JUMP(BPF_JMP | BPF_JSET | BPF_K, SECCOMP_FILTER_FLAG_NEW_LISTENER, 0, 1),
      BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA)),
      BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW),
  };
  sock_fprog fp{(unsigned short)p.size(), p.data()};
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) return os_error("PR_SET_NO_NEW_PRIVS");
  const long fd = syscall(SYS_seccomp, SECCOMP_SET_MODE_FILTER,
                          SECCOMP_FILTER_FLAG_NEW_LISTENER | SECCOMP_FILTER_FLAG_TSYNC | SECCOMP_FILTER_FLAG_TSYNC_ESRCH,
                          &fp);
  if (fd < 0) return os_error("seccomp (listener guard)");
  fcntl((int)fd, F_SETFD, FD_CLOEXEC);
  return PyLong_FromLong(fd);
}

// send_fd(sock, data, fd): `data` on the stream socket `sock`, with
// descriptor `fd` (SCM_RIGHTS) on its first byte
PyObject* py_send_fd(PyObject*, PyObject* args) {
  int sock = -1, fd = -1;
  Py_buffer data;
  if (!PyArg_ParseTuple(args, "iy*i", &sock, &data, &fd)) return nullptr;
  const char* b = (const char*)data.buf;
  size_t left = (size_t)data.len;
  bool first = true;
  while (left > 0) {
    iovec iov{(void*)b, left};
    msghdr mh{};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
    if (first) {
      mh.msg_control = cbuf;
      mh.msg_controllen = sizeof cbuf;
      cmsghdr* cm = CMSG_FIRSTHDR(&mh);
      cm->cmsg_level = SOL_SOCKET;
      cm->cmsg_type = SCM_RIGHTS;
      cm->cmsg_len = CMSG_LEN(sizeof(int));
      memcpy(CMSG_DATA(cm), &fd, sizeof fd);
    }
    const ssize_t n = sendmsg(sock, &mh, MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EINTR) continue;
      PyBuffer_Release(&data);
      return os_error("sendmsg");
    }
    first = false;
    b += n;
    left -= (size_t)n;
  }
  PyBuffer_Release(&data);
  Py_RETURN_NONE;
}

PyObject* py_denied_syscalls(PyObject*, PyObject*) {
  PyObject* l = PyList_New(0);
  for (int nr : kDenied) {
    PyObject* v = PyLong_FromLong(nr);
    PyList_Append(l, v);
    Py_DECREF(v);
  }
  return l;
}

PyMethodDef kMethods[] = {
    {"probe", py_probe, METH_NOARGS, "probe() -> dict: Landlock ABI, seccomp, privilege"},
    {"prepare", py_prepare, METH_VARARGS, "prepare([(path, access), ...]) -> n: open the static Landlock rules"},
    {"apply", py_apply, METH_VARARGS, "apply(opts) -> dict: jail the calling (freshly forked) process"},
    {"denied_syscalls", py_denied_syscalls, METH_NOARGS, "syscall numbers the seccomp filter refuses"},
    {"listen_guard", py_listen_guard, METH_NOARGS,
     "listen_guard() -> fd: hand this sandbox's accept() calls to the daemon (seccomp user notifications)"},
    {"send_fd", py_send_fd, METH_VARARGS, "send_fd(sock, data, fd): data with a descriptor (SCM_RIGHTS)"},
    {"seal_zygote", py_seal_zygote, METH_NOARGS, "install the seccomp filter on the calling zygote (inherited)"},
    {"seal_zygote_net", py_seal_zygote_net, METH_VARARGS,
     "seal_zygote_net([port, ...]) -> dict: Landlock TCP layer denying those ports (inherited)"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_jail", "Sandbox isolation: uid drop, Landlock, seccomp, rlimits.", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__jail() {
  PyObject* m = PyModule_Create(&kModule);
  if (!m) return nullptr;
  PyModule_AddIntConstant(m, "READ", (long)kRead);
  PyModule_AddIntConstant(m, "READ_FILE", (long)LANDLOCK_ACCESS_FS_READ_FILE);
  PyModule_AddIntConstant(m, "WRITE_FILE", (long)LANDLOCK_ACCESS_FS_WRITE_FILE);
  PyModule_AddIntConstant(m, "READ_DIR", (long)LANDLOCK_ACCESS_FS_READ_DIR);
  PyModule_AddIntConstant(m, "TRUNCATE", (long)kFsTruncate);
  PyModule_AddIntConstant(m, "ALL", (long)(kFsV1 | kFsRefer | kFsTruncate));
  return m;
}
