#include "cgroup2.hpp"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace bee {
namespace cg2 {
namespace {

constexpr long kCgroup2Magic = 0x63677270;  // CGROUP2_SUPER_MAGIC

std::string read_text(const std::string& path) {
  std::ifstream f(path);
  if (!f) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

bool has_word(const std::string& text, const char* w) {
  std::istringstream is(text);
  std::string t;
  while (is >> t)
    if (t == w) return true;
  return false;
}

// "key value" lines (memory.events, pids.events)
int64_t event_count(const std::string& path, const char* key) {
  std::istringstream is(read_text(path));
  std::string k;
  int64_t v;
  while (is >> k >> v)
    if (k == key) return v;
  return 0;
}

// this process's cgroup v2 path ("0::/a/b"), "" under v1 / hybrid-only
std::string own_cgroup() {
  std::istringstream is(read_text("/proc/self/cgroup"));
  std::string line;
  while (std::getline(is, line))
    if (line.rfind("0::", 0) == 0) return line.substr(3);
  return "";
}

}  // namespace

bool Manager::write_file(const std::string& path, const std::string& text, std::string* err) const {
  const int fd = open(path.c_str(), O_WRONLY | O_CLOEXEC | (fake_ ? O_CREAT | O_TRUNC : 0), 0644);
  if (fd < 0) {
    if (err) *err = path + ": " + strerror(errno);
    return false;
  }
  const ssize_t n = write(fd, text.data(), text.size());
  const int e = errno;
  close(fd);
  if (n != (ssize_t)text.size()) {
    if (err) *err = path + ": " + strerror(n < 0 ? e : EIO);
    return false;
  }
  return true;
}

bool Manager::init(const std::string& mode, const std::string& root, std::string* why) {
  enabled_ = false;
  fake_ = mode == "fake";
  if (mode == "off") {
    *why = "disabled (--cgroup=off)";
    return false;
  }
  if (mode != "auto" && mode != "require" && !fake_) {
    *why = "unknown --cgroup mode '" + mode + "' (auto, require, off, fake)";
    return false;
  }
  if (fake_ && root.empty()) {
    *why = "--cgroup=fake needs --cgroup-root";
    return false;
  }
  std::string base = root;
  if (base.empty()) {
    const std::string own = own_cgroup();
    if (own.empty()) {
      *why = "no cgroup v2 hierarchy for this process (cgroup v1 or hybrid)";
      return false;
    }
    base = "/sys/fs/cgroup" + (own == "/" ? std::string() : own);
  }
  if (!fake_) {
    struct statfs sf;
    if (statfs(base.c_str(), &sf) != 0 || (long)sf.f_type != kCgroup2Magic) {
      *why = base + " is not a cgroup v2 directory";
      return false;
    }
  }
  if (access(base.c_str(), W_OK) != 0) {
    *why = base + " is not writable by uid " + std::to_string(getuid()) + " (no delegated cgroup v2 subtree)";
    return false;
  }
  const std::string controllers = read_text(base + "/cgroup.controllers");
  if (!has_word(controllers, "memory") || !has_word(controllers, "pids")) {
    *why = base + ": the memory and pids controllers are not available (cgroup.controllers: '" + controllers + "')";
    return false;
  }
  // the leaves need the controllers enabled below `base`; a cgroup with
  // processes of its own cannot enable them (no internal processes), so a
  // delegated directory holds the executor elsewhere or is empty
  std::string sub = read_text(base + "/cgroup.subtree_control");
  if (!has_word(sub, "memory") || !has_word(sub, "pids")) {
    std::string err;
    const std::string want = std::string("+memory +pids") + (has_word(controllers, "cpu") ? " +cpu" : "");
    if (!write_file(base + "/cgroup.subtree_control", fake_ ? "memory pids cpu" : want, &err)) {
      *why = "cannot enable controllers below " + base + " (" + err +
             "): delegate an empty directory and pass it as --cgroup-root";
      return false;
    }
  }
  base_ = base;
  prefix_ = "bee-" + std::to_string(getpid()) + "-";
  enabled_ = true;
  why->clear();
  return true;
}

std::string Manager::create(const std::string& id, const Limits& l, std::string* err) {
  if (!enabled_) return "";
  const std::string leaf = base_ + "/" + prefix_ + id;
  if (mkdir(leaf.c_str(), 0755) != 0 && errno != EEXIST) {
    *err = leaf + ": " + strerror(errno);
    return "";
  }
  bool ok = true;
  if (l.mem_bytes > 0) {
    ok = ok && write_file(leaf + "/memory.max", std::to_string(l.mem_bytes), err);
    if (fake_ || access((leaf + "/memory.swap.max").c_str(), F_OK) == 0)
      ok = ok && write_file(leaf + "/memory.swap.max", "0", err);
    if (fake_ || access((leaf + "/memory.oom.group").c_str(), F_OK) == 0)
      ok = ok && write_file(leaf + "/memory.oom.group", "1", err);
  }
  if (l.tasks > 0) ok = ok && write_file(leaf + "/pids.max", std::to_string(l.tasks), err);
  if (l.cpus > 0 && (fake_ || access((leaf + "/cpu.max").c_str(), F_OK) == 0)) {
    const long period = 100000;
    ok = ok && write_file(leaf + "/cpu.max", std::to_string(std::lround(l.cpus * period)) + " " + std::to_string(period), err);
  }
  if (!ok) {
    remove(leaf);
    return "";
  }
  return leaf;
}

bool Manager::attach(const std::string& leaf, pid_t pid, std::string* err) {
  return write_file(leaf + "/cgroup.procs", std::to_string(pid), err);
}

int64_t Manager::oom_kills(const std::string& leaf) const { return event_count(leaf + "/memory.events", "oom_kill"); }

int64_t Manager::pids_refused(const std::string& leaf) const { return event_count(leaf + "/pids.events", "max"); }

void Manager::kill_all(const std::string& leaf) {
  // (fake: cgroup.procs is only a record of what was attached -- those pids
  // may already belong to other processes)
  if (leaf.empty() || fake_) return;
  if (access((leaf + "/cgroup.kill").c_str(), F_OK) == 0 && write_file(leaf + "/cgroup.kill", "1", nullptr))
    return;
  // kernels before 5.14: every pid listed, a few rounds (a fork can race
  // the walk; pids.max bounds how many)
  for (int round = 0; round < 8; ++round) {
    std::istringstream is(read_text(leaf + "/cgroup.procs"));
    pid_t p;
    int n = 0;
    while (is >> p)
      if (p > 0 && p != getpid()) {
        kill(p, SIGKILL);
        ++n;
      }
    if (n == 0) break;
  }
}

bool Manager::remove(const std::string& leaf) {
  if (leaf.empty()) return true;
  if (fake_) {
    // the "interface files" of a plain directory are files of ours
    if (DIR* d = opendir(leaf.c_str())) {
      while (dirent* e = readdir(d))
        if (e->d_name[0] != '.') unlink((leaf + "/" + e->d_name).c_str());
      closedir(d);
    }
  }
  return rmdir(leaf.c_str()) == 0 || errno == ENOENT;
}

}  // namespace cg2
}  // namespace bee
