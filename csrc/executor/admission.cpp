#include "admission.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>

namespace bee {

double Admission::now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Admission::Admission(AdmissionLimits lim) : lim_(lim) {}

Admission::~Admission() { unmap_load_table(); }

bool Admission::map_load_table(const std::string& path, std::string* err) {
  const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC | O_NOFOLLOW, 0600);
  if (fd < 0) {
    if (err) *err = strerror(errno);
    return false;
  }
  void* m = MAP_FAILED;
  if (ftruncate(fd, 4096) == 0) m = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  const int e = errno;
  close(fd);
  if (m == MAP_FAILED) {
    unlink(path.c_str());
    if (err) *err = strerror(e);
    return false;
  }
  std::lock_guard<std::mutex> lk(mu_);
  load_ = static_cast<LoadTable*>(m);
  load_path_ = path;
  publish_locked();
  return true;
}

void Admission::unmap_load_table() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!load_) return;
  munmap(load_, 4096);
  load_ = nullptr;
  unlink(load_path_.c_str());
}

std::string Admission::refuse_reason(const JobClaim& c) const {
  // a gang's rank takes the place of the warm rank it runs as: while it runs,
  // that rank's standing charge is its own HBM, not an extra (a gang holds
  // its slots reserved, so nothing else is admitted beside it meanwhile)
  const bool gang = c.ranks > 1;
  const int64_t hbm_standing = std::max<int64_t>(lim_.standing_hbm - (gang ? lim_.standing_rank_hbm : 0), 0);
  const int64_t hbm_room = lim_.hbm_capacity - hbm_standing;
  if (lim_.hbm_capacity > 0 && c.hbm > hbm_room)
    return "hbm_quota of " + std::to_string(c.hbm >> 20) + " MiB exceeds this GPU's usable HBM (" +
           std::to_string(std::max<int64_t>(hbm_room, 0) >> 20) + " MiB" +
           (hbm_standing > 0 ? " after " + std::to_string(hbm_standing >> 20) + " MiB held by warm gang ranks"
                             : std::string()) +
           ")";
  // a gang's ranks run on as many slots, each drained for it: N shares
  const int64_t ranks = std::max(1, c.ranks);
  const int64_t mem_standing = std::max<int64_t>(lim_.standing_mem - (gang ? lim_.standing_rank_mem : 0), 0);
  const int64_t mem_room = (lim_.mem_capacity - mem_standing) * ranks;
  if (lim_.mem_capacity > 0 && c.mem > mem_room)
    return "the job's sandbox memory bound (" + std::to_string(c.mem >> 20) + " MiB) exceeds its slots' " +
           "host-memory capacity (" + std::to_string(std::max<int64_t>(mem_room, 0) >> 20) + " MiB)";
  return std::string();
}

bool Admission::fits_locked(const JobClaim& c) const {
  if (c.bypass) return true;
  return (lim_.max_inflight <= 0 || jobs_ < lim_.max_inflight) &&
         (lim_.hbm_capacity <= 0 || lim_.standing_hbm + hbm_committed_ + c.hbm <= lim_.hbm_capacity) &&
         (lim_.mem_capacity <= 0 || lim_.standing_mem + mem_committed_ + c.mem <= lim_.mem_capacity);
}

bool Admission::held_locked(const JobClaim& c) const { return !c.bypass && reserved_ && now_ms() < reserved_until_; }

AdmitStatus Admission::admit(const JobClaim& c, bool try_only, const std::atomic<bool>* stopping) {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t ticket = next_ticket_++;
  queue_.push_back(ticket);
  publish_locked();
  auto leave = [&] {
    for (auto it = queue_.begin(); it != queue_.end(); ++it)
      if (*it == ticket) {
        queue_.erase(it);
        break;
      }
    publish_locked();
  };
  const double deadline = now_ms() + lim_.timeout_s * 1e3;
  while (true) {
    const bool held = held_locked(c);
    if (!held && fits_locked(c) && (c.bypass || queue_.front() == ticket)) break;
    if (stopping && stopping->load()) {
      leave();
      return AdmitStatus::kStopping;
    }
    if (try_only) {
      leave();
      busy_++;
      return held ? AdmitStatus::kReserved : AdmitStatus::kBusy;
    }
    const double left = deadline - now_ms();
    if (left <= 0) {
      leave();
      timeouts_++;
      lk.unlock();
      cv_.notify_all();  // (the tickets behind this one may move up)
      return AdmitStatus::kTimeout;
    }
    // woken by every finish / release; the 50 ms bound also catches a
    // reservation's TTL running out and `stopping`
    cv_.wait_for(lk, std::chrono::milliseconds((int64_t)std::min(left, 50.0) + 1));
  }
  leave();
  jobs_++;
  admitted_++;
  hbm_committed_ += c.hbm;
  mem_committed_ += c.mem;
  max_jobs_seen_ = std::max(max_jobs_seen_, jobs_);
  max_hbm_seen_ = std::max(max_hbm_seen_, hbm_committed_);
  max_mem_seen_ = std::max(max_mem_seen_, mem_committed_);
  publish_locked();
  lk.unlock();
  cv_.notify_all();  // the next ticket may fit as well
  return AdmitStatus::kAdmitted;
}

void Admission::finish(const JobClaim& c) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    jobs_--;
    hbm_committed_ -= c.hbm;
    mem_committed_ -= c.mem;
    publish_locked();
  }
  cv_.notify_all();
}

bool Admission::reserve(double ttl_s, double wait_s, const std::atomic<bool>* stopping) {
  std::unique_lock<std::mutex> lk(mu_);
  reserved_ = true;
  reserved_until_ = now_ms() + ttl_s * 1e3;
  publish_locked();
  const double deadline = now_ms() + wait_s * 1e3;
  while (jobs_ > 0 && now_ms() < deadline && !(stopping && stopping->load()))
    cv_.wait_for(lk, std::chrono::milliseconds(20));
  return jobs_ == 0;
}

void Admission::release() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    reserved_ = false;
    publish_locked();
  }
  cv_.notify_all();
}

void Admission::wake_all() { cv_.notify_all(); }

AdmissionSnapshot Admission::snapshot() const {
  std::lock_guard<std::mutex> lk(mu_);
  AdmissionSnapshot s;
  s.jobs = jobs_;
  s.waiting = (int64_t)queue_.size();
  s.hbm_committed = hbm_committed_;
  s.mem_committed = mem_committed_;
  s.admitted = admitted_;
  s.max_jobs_seen = max_jobs_seen_;
  s.max_hbm_seen = max_hbm_seen_;
  s.max_mem_seen = max_mem_seen_;
  s.busy = busy_;
  s.timeouts = timeouts_;
  s.reserved = reserved_ && now_ms() < reserved_until_;
  return s;
}

void Admission::publish_locked() {
  if (!load_) return;
  LoadTable* t = load_;
  __atomic_store_n(&t->seq, t->seq + 1, __ATOMIC_RELEASE);  // odd: being written
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  t->magic = kLoadMagic;
  t->jobs = jobs_;
  t->waiting = (int64_t)queue_.size();
  // the routing view of HBM headroom: what jobs committed plus what idle
  // warm gang ranks hold
  t->hbm_committed = hbm_committed_ + lim_.standing_hbm;
  t->max_inflight = lim_.max_inflight;
  t->hbm_capacity = lim_.hbm_capacity;
  t->reserved = reserved_ && now_ms() < reserved_until_ ? 1 : 0;
  t->executions = admitted_;
  t->pid = getpid();
  t->max_jobs_seen = max_jobs_seen_;
  t->max_hbm_seen = max_hbm_seen_;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  __atomic_store_n(&t->seq, t->seq + 1, __ATOMIC_RELEASE);
}

}  // namespace bee
