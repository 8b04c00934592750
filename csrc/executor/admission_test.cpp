// CPU unit test of the admission state machine (admission.hpp): tickets in
// arrival order, the in-flight / HBM / host-memory bounds, standing
// commitments, try-only answers, time-outs, gang reservations with their TTL
// and bypass, and a many-thread stress run -- no daemon, no service harness.
// Built under ThreadSanitizer by _build.py ("admission-test"); driven by
// tests/test_admission_unit_cpu.py, which checks the exit status and the
// per-case lines.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "admission.hpp"

using namespace bee;

namespace {

int g_failed = 0;

#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
      ++g_failed;                                                          \
    }                                                                      \
  } while (0)

void sleep_ms(int ms) { std::this_thread::sleep_for(std::chrono::milliseconds(ms)); }

AdmissionLimits limits(int inflight, int64_t hbm = 0, int64_t mem = 0) {
  AdmissionLimits l;
  l.max_inflight = inflight;
  l.hbm_capacity = hbm;
  l.mem_capacity = mem;
  l.timeout_s = 5.0;
  return l;
}

JobClaim claim(int64_t hbm = 0, int64_t mem = 0, bool bypass = false) {
  JobClaim c;
  c.hbm = hbm;
  c.mem = mem;
  c.bypass = bypass;
  return c;
}

// tickets are served in arrival order: with one slot, the jobs that queue
// behind a running one start in the order they arrived
void fifo_order() {
  Admission a(limits(1));
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
  std::mutex mu;
  std::vector<int> order;
  std::vector<std::thread> ts;
  for (int i = 0; i < 5; ++i) {
    ts.emplace_back([&, i] {
      CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
      {
        std::lock_guard<std::mutex> lk(mu);
        order.push_back(i);
      }
      sleep_ms(5);
      a.finish(claim());
    });
    // the next thread arrives only once this one holds its ticket
    while (a.snapshot().waiting < i + 1) sleep_ms(1);
  }
  CHECK(a.snapshot().waiting == 5 && a.snapshot().jobs == 1);
  a.finish(claim());
  for (auto& t : ts) t.join();
  CHECK((order == std::vector<int>{0, 1, 2, 3, 4}));
  const AdmissionSnapshot s = a.snapshot();
  CHECK(s.jobs == 0 && s.waiting == 0 && s.admitted == 6 && s.max_jobs_seen == 1);
}

// HBM quotas commit against the capacity; a job that does not fit waits for
// one that ends; try-only says "busy" at once
void hbm_commitment() {
  Admission a(limits(0, 10 << 20));
  CHECK(a.admit(claim(6 << 20), false, nullptr) == AdmitStatus::kAdmitted);
  CHECK(a.admit(claim(6 << 20), true, nullptr) == AdmitStatus::kBusy);
  CHECK(a.admit(claim(4 << 20), false, nullptr) == AdmitStatus::kAdmitted);  // fits beside it
  std::atomic<bool> admitted{false};
  std::thread t([&] {
    CHECK(a.admit(claim(6 << 20), false, nullptr) == AdmitStatus::kAdmitted);
    admitted = true;
  });
  sleep_ms(60);
  CHECK(!admitted.load());
  a.finish(claim(6 << 20));
  t.join();
  CHECK(admitted.load());
  const AdmissionSnapshot s = a.snapshot();
  CHECK(s.hbm_committed == (10 << 20) && s.max_hbm_seen == (10 << 20) && s.busy == 1);
  a.finish(claim(4 << 20));
  a.finish(claim(6 << 20));
  CHECK(a.snapshot().hbm_committed == 0);
}

// host memory commits the same way, per slot share
void mem_commitment() {
  Admission a(limits(0, 0, 8 << 20));
  CHECK(a.admit(claim(0, 5 << 20), false, nullptr) == AdmitStatus::kAdmitted);
  CHECK(a.admit(claim(0, 4 << 20), true, nullptr) == AdmitStatus::kBusy);
  CHECK(a.admit(claim(0, 3 << 20), true, nullptr) == AdmitStatus::kAdmitted);
  CHECK(a.snapshot().mem_committed == (8 << 20));
  a.finish(claim(0, 5 << 20));
  a.finish(claim(0, 3 << 20));
}

// idle warm gang ranks hold HBM and host memory: charged up front, so a job
// that fits the GPU but not what they leave is refused (never admissible)
// and the room left is what they leave
void standing_commitments() {
  AdmissionLimits l = limits(0, 10 << 20, 10 << 20);
  l.standing_hbm = 3 << 20;
  l.standing_mem = 2 << 20;
  Admission a(l);
  CHECK(!a.refuse_reason(claim(8 << 20)).empty());
  CHECK(a.refuse_reason(claim(8 << 20)).find("warm gang ranks") != std::string::npos);
  CHECK(a.refuse_reason(claim(7 << 20)).empty());
  CHECK(!a.refuse_reason(claim(0, 9 << 20)).empty());
  JobClaim gang = claim(0, 16 << 20);
  gang.ranks = 2;  // a 2-rank gang's memory spreads over two slots' shares
  CHECK(a.refuse_reason(gang).empty());
  CHECK(a.admit(claim(7 << 20), false, nullptr) == AdmitStatus::kAdmitted);
  CHECK(a.admit(claim(1 << 20), true, nullptr) == AdmitStatus::kBusy);  // 3 + 7 + 1 > 10
  a.finish(claim(7 << 20));
}

// a gang's rank runs as the warm rank it takes: its claim may use that rank's
// share of the standing charge (counted once, not twice), a single job not
void gang_rank_replaces_warm_rank() {
  AdmissionLimits l = limits(0, 10 << 20, 10 << 20);
  l.standing_hbm = 3 << 20;  // three warm ranks of 1 MiB
  l.standing_mem = 3 << 20;
  l.standing_rank_hbm = 1 << 20;
  l.standing_rank_mem = 1 << 20;
  Admission a(l);
  JobClaim one = claim(8 << 20);
  CHECK(!a.refuse_reason(one).empty());  // 8 > 10 - 3
  JobClaim rank = claim(8 << 20);
  rank.ranks = 2;
  CHECK(a.refuse_reason(rank).empty());  // 8 <= 10 - (3 - 1)
  rank.hbm = 9 << 20;
  CHECK(a.refuse_reason(rank).find("2 MiB held by warm gang ranks") != std::string::npos);
  JobClaim mem = claim(0, 16 << 20);
  mem.ranks = 2;  // (10 - 2) x 2 ranks
  CHECK(a.refuse_reason(mem).empty());
  mem.mem = 17 << 20;
  CHECK(!a.refuse_reason(mem).empty());
}

// a waiting job gives up at its deadline, and the tickets behind it move up
void timeout() {
  AdmissionLimits l = limits(1);
  l.timeout_s = 0.1;
  Admission a(l);
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
  const double t0 = Admission::now_ms();
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kTimeout);
  const double waited = Admission::now_ms() - t0;
  CHECK(waited >= 90 && waited < 1000);
  const AdmissionSnapshot s = a.snapshot();
  CHECK(s.timeouts == 1 && s.waiting == 0);
  a.finish(claim());
}

// a gang reservation holds new jobs back (try-only: "reserved"), drains the
// running ones, lets the gang's own job through, and lapses at its TTL when
// nobody releases it (a front-end that died)
void reservation() {
  Admission a(limits(4));
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
  std::atomic<bool> drained{false};
  std::thread r([&] { drained = a.reserve(10.0, 2.0, nullptr); });
  while (!a.snapshot().reserved) sleep_ms(1);
  CHECK(a.admit(claim(), true, nullptr) == AdmitStatus::kReserved);
  sleep_ms(30);
  CHECK(!drained.load());
  a.finish(claim());
  r.join();
  CHECK(drained.load());
  CHECK(a.admit(claim(0, 0, true), false, nullptr) == AdmitStatus::kAdmitted);  // the gang's job
  std::atomic<bool> waiter_in{false};
  std::thread w([&] {
    CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
    waiter_in = true;
  });
  sleep_ms(60);
  CHECK(!waiter_in.load());
  a.release();
  w.join();
  CHECK(waiter_in.load());
  a.finish(claim(0, 0, true));
  a.finish(claim());
  // TTL: a reservation nobody releases
  CHECK(a.reserve(0.15, 0.0, nullptr));
  const double t0 = Admission::now_ms();
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
  CHECK(Admission::now_ms() - t0 >= 100);
  CHECK(!a.snapshot().reserved);
  a.finish(claim());
}

// shutdown: waiters return "stopping"
void stopping() {
  Admission a(limits(1));
  CHECK(a.admit(claim(), false, nullptr) == AdmitStatus::kAdmitted);
  std::atomic<bool> stop{false};
  AdmitStatus got = AdmitStatus::kAdmitted;
  std::thread t([&] { got = a.admit(claim(), false, &stop); });
  while (a.snapshot().waiting < 1) sleep_ms(1);
  stop = true;
  a.wake_all();
  t.join();
  CHECK(got == AdmitStatus::kStopping);
  a.finish(claim());
}

// many threads, bounds never exceeded, every job admitted once, nothing left
void stress() {
  Admission a(limits(3, 64 << 20));
  std::atomic<int> running{0}, peak{0}, done{0};
  std::atomic<int64_t> hbm{0};
  std::atomic<bool> over{false};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) {
    ts.emplace_back([&, t] {
      for (int i = 0; i < 150; ++i) {
        const JobClaim c = claim((int64_t)(1 + (t + i) % 24) << 20);
        if (a.admit(c, false, nullptr) != AdmitStatus::kAdmitted) {
          over = true;
          continue;
        }
        const int now = ++running;
        int p = peak.load();
        while (now > p && !peak.compare_exchange_weak(p, now)) {
        }
        if ((hbm += c.hbm) > (64 << 20)) over = true;
        // hold the job a moment: with a bare yield, a loaded CPU (the suite
        // under TSan) could run the threads one after another and never
        // overlap two jobs
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        hbm -= c.hbm;
        --running;
        a.finish(c);
        ++done;
      }
    });
  }
  for (auto& t : ts) t.join();
  CHECK(!over.load());
  CHECK(peak.load() <= 3 && peak.load() >= 2);
  CHECK(done.load() == 8 * 150);
  const AdmissionSnapshot s = a.snapshot();
  CHECK(s.jobs == 0 && s.waiting == 0 && s.hbm_committed == 0 && s.admitted == 8 * 150);
  CHECK(s.max_jobs_seen <= 3 && s.max_hbm_seen <= (64 << 20));
}

// the load table front-end replicas read: seqlock even after every write,
// standing HBM counted in the routing view
void load_table(const char* dir) {
  AdmissionLimits l = limits(2, 100 << 20);
  l.standing_hbm = 5 << 20;
  Admission a(l);
  const std::string path = std::string(dir) + "/load-test";
  std::string err;
  CHECK(a.map_load_table(path, &err));
  CHECK(a.admit(claim(10 << 20), false, nullptr) == AdmitStatus::kAdmitted);
  FILE* f = std::fopen(path.c_str(), "rb");
  CHECK(f != nullptr);
  if (f) {
    LoadTable t{};
    CHECK(std::fread(&t, sizeof t, 1, f) == 1);
    std::fclose(f);
    CHECK(t.magic == kLoadMagic && t.seq % 2 == 0);
    CHECK(t.jobs == 1 && t.hbm_committed == (15 << 20) && t.max_inflight == 2 && t.executions == 1);
  }
  a.finish(claim(10 << 20));
  a.unmap_load_table();
  CHECK(std::fopen(path.c_str(), "rb") == nullptr);
}

}  // namespace

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  struct Case {
    const char* name;
    void (*fn)();
  } cases[] = {{"fifo_order", fifo_order},       {"hbm_commitment", hbm_commitment},
               {"mem_commitment", mem_commitment}, {"standing_commitments", standing_commitments},
               {"gang_rank_replaces_warm_rank", gang_rank_replaces_warm_rank},
               {"timeout", timeout},             {"reservation", reservation},
               {"stopping", stopping},           {"stress", stress}};
  for (auto& c : cases) {
    const int before = g_failed;
    c.fn();
    std::printf("%s %s\n", g_failed == before ? "PASS" : "FAIL", c.name);
  }
  {
    const int before = g_failed;
    load_table(dir);
    std::printf("%s load_table\n", g_failed == before ? "PASS" : "FAIL");
  }
  std::fflush(stdout);
  return g_failed == 0 ? 0 : 1;
}
