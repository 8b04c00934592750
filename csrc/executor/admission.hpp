// Admission of jobs on one GPU slot, shared by every front-end replica of
// the node (they all send this GPU's jobs to its daemon): at most
// max_inflight admitted jobs, their HBM quotas within the GPU's capacity and
// their sandbox trees' memory bounds within the slot's share of host memory;
// the rest wait in arrival order (tickets), or get a "busy" answer when they
// asked not to wait.  A gang reservation holds new jobs back and drains the
// running ones; the gang's own job bypasses both.
//
// Standing commitments: idle warm gang rank sets (sandbox_gang.cpp) hold a
// HIP context and torch's state on this GPU and their host memory whether or
// not a job runs, so they are charged against the capacities up front.
//
// Self-contained (no HIP, no pool): the CPU unit test (admission_test.cpp,
// tests/test_admission_unit_cpu.py) drives it directly.  The reference has no
// admission at all: every Execute gets a pod, spawning one synchronously when
// the pool is empty (kubernetes_code_executor.py:268-272).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>

namespace bee {

// Load of one daemon, published in a small shared file (<run_dir>/load-<pid>)
// that front-end replicas map read-only: they route each request to the
// least-loaded GPU as seen by all replicas, not by their own requests alone
// (scheduler/local_gpu_pool.py).  Seqlock: `seq` is odd while it is written.
struct LoadTable {
  uint64_t magic;  // kLoadMagic
  uint64_t seq;
  int64_t jobs;           // admitted, running
  int64_t waiting;        // waiting for admission
  int64_t hbm_committed;  // HBM quotas of the admitted jobs (+ the standing commitments)
  int64_t max_inflight;
  int64_t hbm_capacity;
  int64_t reserved;       // 1 while a gang holds this GPU
  int64_t executions;     // admitted since start
  int64_t pid;
  int64_t max_jobs_seen;  // high-water marks (what the admission bound held to)
  int64_t max_hbm_seen;
};
constexpr uint64_t kLoadMagic = 0x3130444f4c454542ull;  // "BEELOD01" little endian

struct AdmissionLimits {
  int max_inflight = 0;       // 0 = unbounded
  int64_t hbm_capacity = 0;   // bytes of this GPU jobs may commit; 0 = unbounded
  int64_t mem_capacity = 0;   // bytes of host memory for this slot's sandbox trees; 0 = unbounded
  int64_t standing_hbm = 0;   // held by idle warm gang ranks on this GPU
  int64_t standing_mem = 0;
  // one warm rank's share of them: a gang's rank runs as (replaces) the warm
  // rank it takes, so a gang claim may use that rank's room too
  int64_t standing_rank_hbm = 0;
  int64_t standing_rank_mem = 0;
  double timeout_s = 900.0;   // longest wait for admission
};

struct JobClaim {
  int64_t hbm = 0;      // the job's HBM quota on this GPU
  int64_t mem = 0;      // its sandbox trees' host-memory bound
  int ranks = 1;        // a gang's ranks run on as many slots (each drained for it)
  bool bypass = false;  // the job of the gang holding the reservation
};

enum class AdmitStatus { kAdmitted, kBusy, kReserved, kTimeout, kStopping };

struct AdmissionSnapshot {
  int64_t jobs = 0, waiting = 0, hbm_committed = 0, mem_committed = 0, admitted = 0;
  int64_t max_jobs_seen = 0, max_hbm_seen = 0, max_mem_seen = 0, busy = 0, timeouts = 0;
  bool reserved = false;
};

class Admission {
 public:
  explicit Admission(AdmissionLimits lim);
  ~Admission();
  Admission(const Admission&) = delete;
  Admission& operator=(const Admission&) = delete;

  // publish the load table at `path` (created 0600); false if unavailable
  bool map_load_table(const std::string& path, std::string* err);
  void unmap_load_table();
  const std::string& load_path() const { return load_path_; }
  bool load_mapped() const { return load_ != nullptr; }

  // why a claim can never be admitted here ("" = it can): quotas beyond the
  // capacities left after the standing commitments
  std::string refuse_reason(const JobClaim& c) const;
  // take a ticket and wait, in arrival order, until the claim fits (a
  // bypassing claim only waits for nothing); try_only: kBusy / kReserved at
  // once instead of waiting; `stopping` checked while waiting
  AdmitStatus admit(const JobClaim& c, bool try_only, const std::atomic<bool>* stopping);
  void finish(const JobClaim& c);  // an admitted job ended: its commitments are free again

  // gang reservation: hold new jobs back for ttl_s; true once no admitted
  // job runs (within wait_s)
  bool reserve(double ttl_s, double wait_s, const std::atomic<bool>* stopping);
  void release();
  void wake_all();  // (shutdown: waiters re-check `stopping`)

  AdmissionSnapshot snapshot() const;
  const AdmissionLimits& limits() const { return lim_; }

  static double now_ms();

 private:
  bool fits_locked(const JobClaim& c) const;
  bool held_locked(const JobClaim& c) const;
  void publish_locked();

  AdmissionLimits lim_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  int64_t jobs_ = 0, hbm_committed_ = 0, mem_committed_ = 0, admitted_ = 0;
  int64_t max_jobs_seen_ = 0, max_hbm_seen_ = 0, max_mem_seen_ = 0, busy_ = 0, timeouts_ = 0;
  uint64_t next_ticket_ = 0;
  std::deque<uint64_t> queue_;  // waiting tickets, in arrival order
  bool reserved_ = false;
  double reserved_until_ = 0;  // now_ms() clock
  LoadTable* load_ = nullptr;
  std::string load_path_;
};

}  // namespace bee
