#include "procmon.hpp"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>

namespace bee {
namespace procmon {

namespace {

// small /proc files: one read
ssize_t read_small(const char* path, char* buf, size_t cap) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  ssize_t n = 0;
  while ((size_t)n < cap - 1) {
    const ssize_t r = read(fd, buf + n, cap - 1 - (size_t)n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    n += r;
  }
  close(fd);
  buf[n > 0 ? n : 0] = 0;
  return n;
}

// "Key:   1234 kB" -> bytes; -1 when the key is absent
int64_t kb_field(const char* text, const char* key) {
  const char* p = strstr(text, key);
  while (p && p != text && p[-1] != '\n') p = strstr(p + 1, key);
  if (!p) return -1;
  return strtoll(p + strlen(key), nullptr, 10) * 1024;
}

void children_of(pid_t pid, std::vector<pid_t>* out) {
  char task[64];
  snprintf(task, sizeof task, "/proc/%d/task", (int)pid);
  DIR* d = opendir(task);
  if (!d) return;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    char path[128], buf[8192];
    snprintf(path, sizeof path, "/proc/%d/task/%s/children", (int)pid, e->d_name);
    if (read_small(path, buf, sizeof buf) <= 0) continue;
    for (char* p = buf; *p;) {
      char* end;
      const long c = strtol(p, &end, 10);
      if (end == p) break;
      out->push_back((pid_t)c);
      p = end;
      while (*p == ' ' || *p == '\n') ++p;
    }
  }
  closedir(d);
}

}  // namespace

void tree(pid_t leader, std::vector<pid_t>* out, size_t cap) {
  out->clear();
  if (leader <= 0) return;
  std::vector<pid_t> kids;
  out->push_back(leader);
  for (size_t i = 0; i < out->size() && out->size() < cap; ++i) {
    kids.clear();
    children_of((*out)[i], &kids);
    for (pid_t k : kids) {
      if (out->size() >= cap) break;
      out->push_back(k);
    }
  }
}

Sample sample(pid_t pid) {
  Sample s;
  char path[64], buf[4096];
  snprintf(path, sizeof path, "/proc/%d/stat", (int)pid);
  if (read_small(path, buf, sizeof buf) <= 0) return s;
  const char* rp = strrchr(buf, ')');  // comm may hold spaces and parens
  if (!rp) return s;
  // fields after the comm: state(3) ... utime(14) stime(15) cutime(16) cstime(17) ... num_threads(20)
  char state = 0;
  unsigned long long f[18] = {0};
  int got = sscanf(rp + 1, " %c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %llu %llu %llu %llu %*d %*d %llu", &state,
                   &f[0], &f[1], &f[2], &f[3], &f[4]);
  if (got < 6) return s;
  if (state == 'Z' || state == 'X') return s;  // exited: nothing resident, reaped time lands in its parent
  static const double tck = (double)sysconf(_SC_CLK_TCK);
  s.cpu_ms = (double)(f[0] + f[1] + f[2] + f[3]) * 1e3 / tck;
  s.tasks = (int64_t)f[4];
  snprintf(path, sizeof path, "/proc/%d/status", (int)pid);
  if (read_small(path, buf, sizeof buf) > 0) {
    const int64_t anon = kb_field(buf, "RssAnon:"), shmem = kb_field(buf, "RssShmem:");
    s.anon_bytes = (anon > 0 ? anon : 0) + (shmem > 0 ? shmem : 0);
  }
  s.alive = true;
  return s;
}

int64_t pss_anon_bytes(pid_t pid) {
  char path[64], buf[4096];
  snprintf(path, sizeof path, "/proc/%d/smaps_rollup", (int)pid);
  if (read_small(path, buf, sizeof buf) <= 0) return -1;
  const int64_t a = kb_field(buf, "Pss_Anon:"), sh = kb_field(buf, "Pss_Shmem:");
  if (a >= 0) return a + (sh > 0 ? sh : 0);
  return kb_field(buf, "Pss:");
}

int64_t vram_bytes(pid_t pid, std::set<std::string>* clients, bool* has_render) {
  char fddir[64];
  snprintf(fddir, sizeof fddir, "/proc/%d/fd", (int)pid);
  DIR* d = opendir(fddir);
  if (!d) return 0;
  int64_t total = 0;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    char target[128];
    const ssize_t tl = readlinkat(dirfd(d), e->d_name, target, sizeof target - 1);
    if (tl <= 0) continue;
    target[tl] = 0;
    if (strncmp(target, "/dev/dri/renderD", 16) != 0) continue;
    if (has_render) *has_render = true;
    char ipath[128], info[8192];
    snprintf(ipath, sizeof ipath, "/proc/%d/fdinfo/%s", (int)pid, e->d_name);
    if (read_small(ipath, info, sizeof info) <= 0) continue;
    // dup'd descriptors share one DRM client: count each client once
    const char* cid = strstr(info, "drm-client-id:");
    std::string client = cid ? std::string(cid, strcspn(cid, "\n")) : std::string(e->d_name);
    if (!clients->insert(std::to_string(pid) + "/" + client).second) continue;
    const char* v = strstr(info, "drm-total-vram:");
    if (!v) continue;
    total += (int64_t)strtoll(v + 15, nullptr, 10) * 1024;  // KiB
  }
  closedir(d);
  return total;
}

namespace {

pid_t parent_of(pid_t pid) {
  char path[64], buf[1024];
  snprintf(path, sizeof path, "/proc/%d/stat", (int)pid);
  if (read_small(path, buf, sizeof buf) <= 0) return -1;
  const char* rp = strrchr(buf, ')');
  int ppid = -1;
  if (!rp || sscanf(rp + 1, " %*c %d", &ppid) != 1) return -1;
  return (pid_t)ppid;
}

// Signal `child`, read earlier from `parent`'s children list, only if it is
// still that process: between the read and the signal the child may have
// been reaped and its PID handed to an unrelated process (the daemon is
// privileged enough to signal it).  A pidfd pins the process it was opened
// on; its parent is checked after the open, so a recycled PID (whose parent
// is someone else) is skipped, and a pinned process that dies before the
// signal only makes the signal fail.
bool signal_child(pid_t parent, pid_t child, int sig) {
  const int fd = (int)syscall(SYS_pidfd_open, child, 0);
  if (fd < 0) {
    if (errno != ENOSYS) return false;  // gone already (ESRCH)
    // kernels before pidfd (5.3): best effort, checked the same way
    return parent_of(child) == parent && kill(child, sig) == 0;
  }
  bool ok = parent_of(child) == parent && syscall(SYS_pidfd_send_signal, fd, sig, nullptr, 0) == 0;
  close(fd);
  return ok;
}

// (parent, child) pairs of the tree below `leader`, breadth first
void tree_edges(pid_t leader, std::vector<std::pair<pid_t, pid_t>>* out, size_t cap = 4096) {
  out->clear();
  std::vector<pid_t> frontier{leader}, kids;
  for (size_t i = 0; i < frontier.size() && out->size() < cap; ++i) {
    kids.clear();
    children_of(frontier[i], &kids);
    for (pid_t k : kids) {
      if (out->size() >= cap) break;
      out->emplace_back(frontier[i], k);
      frontier.push_back(k);
    }
  }
}

}  // namespace

int kill_tree(pid_t leader, int rounds) {
  if (leader <= 0) return 0;
  // freeze the leader's process group first (atomic for its members: a fork
  // bomb in it stops growing); a stopped leader still adopts the orphans of
  // what is killed below it
  kill(-leader, SIGSTOP);
  kill(leader, SIGSTOP);
  std::set<pid_t> signalled;
  std::vector<std::pair<pid_t, pid_t>> edges;
  for (int r = 0; r < rounds; ++r) {
    tree_edges(leader, &edges);
    size_t fresh = 0;
    for (auto& e : edges) {
      if (e.second == leader || signalled.count(e.second)) continue;  // (killed ones linger as zombies)
      if (signal_child(e.first, e.second, SIGKILL)) {
        signalled.insert(e.second);
        ++fresh;
      }
    }
    if (!fresh) break;
  }
  kill(-leader, SIGKILL);  // the process group, the leader with it
  kill(leader, SIGKILL);
  return (int)signalled.size() + 1;
}

void signal_tree(pid_t leader, int sig) {
  if (leader <= 0) return;
  kill(-leader, sig);
  kill(leader, sig);
  std::vector<std::pair<pid_t, pid_t>> edges;
  tree_edges(leader, &edges);
  for (auto& e : edges) signal_child(e.first, e.second, sig);
}

}  // namespace procmon
}  // namespace bee
