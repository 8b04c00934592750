// Sandbox pool: single-use Python workers forked from a pre-imported zygote,
// pinned to this executor's GPU, warmed (HIP context + kernel code object)
// while they wait, used for exactly one execution, then destroyed.
//
// Replaces the reference's per-request executor pod + in-pod actix server
// (`executor/server.rs:139-228`, `kubernetes_code_executor.py:163-279`):
// the "pod" becomes a forked process group with a private workspace, the
// pod pool becomes the warm-worker deque, and the per-pod upm/xonsh/python
// cold start (~1.5 s for torch) is paid once by the zygote.
#pragma once
#include <sys/types.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "admission.hpp"
#include "broker_core.hpp"
#include "listen_guard.hpp"
#include "cgroup2.hpp"
#include "json.hpp"

namespace bee {

struct PoolConfig {
  std::string sandbox_root = "/tmp/bee-sandboxes";
  std::string run_dir;                 // control sockets; default <sandbox_root>/.run
  std::string python = "python3";
  std::string zygote_module = "bee_code_interpreter_fs_amd.runtime.zygote";
  std::string gpus;                    // HIP_VISIBLE_DEVICES for pooled workers ("" = CPU only)
  int target = 4;                      // warm workers kept ready
  int max_concurrent_spawns = 8;       // HIP init contends in the driver
  bool warm_gpu = true;
  bool recursive_scan = false;
  int64_t max_output_bytes = 16 << 20;
  double default_timeout_s = 60.0;
  double acquire_timeout_s = 120.0;
  double max_idle_s = 900.0;           // recycle warm sandboxes idle longer than this (0 = never)
  int64_t default_hbm_quota = 0;
  std::string zygote_preload;          // LD_PRELOAD for the zygote (HBM interposer)
  std::map<std::string, std::string> extra_env;
  // pod mode: one fixed sandbox (reference k8s contract)
  bool pod_mode = false;
  std::string pod_workspace = "/workspace";
  std::string pod_runtime_packages = "/runtime-packages";
  std::string pythonpath;              // prepended to PYTHONPATH of zygote
  // kernel broker: the daemon owns the GPU context; "light" sandboxes call
  // beekern through it and never initialise HIP themselves
  std::string broker_lib;              // path of libbeekern.so ("" = no broker)
  int light_target = 8;                // warm light sandboxes kept ready
  int light_zygotes = 2;               // parallel forkers for light sandboxes
  std::string light_preload = "numpy,pandas,scipy.stats,matplotlib.pyplot,PIL.Image,bee_code_interpreter_fs_amd.ops";
  int min_target = 0;                  // warm minimal sandboxes kept ready (0 = no minimal zygotes)
  int min_zygotes = 0;                 // parallel forkers for minimal sandboxes
  int min_cpu_target = -1;             // warm lazy-session minimal sandboxes (-1 = min_target; GPU pools only)
  std::string min_preload = "numpy,numpy.random,bee_code_interpreter_fs_amd.ops";
  int nano_target = 0;                 // warm numpy-free sandboxes kept ready (0 = no nano zygotes)
  int nano_zygotes = 0;                // parallel forkers for nano sandboxes
  int nano_cpu_target = -1;            // warm lazy-session nano sandboxes (-1 = nano_target; GPU pools only)
  std::string nano_preload = "bee_code_interpreter_fs_amd.ops";
  // sandbox jail (csrc/jail, runtime/jail.py): Landlock filesystem view,
  // signal/ptrace/abstract-socket scoping, seccomp, rlimits -- and, when the
  // daemon runs as root and uid_base > 0, a UID/GID of each sandbox's own
  bool jail = false;
  bool listen_guard = true;            // --listen-guard: sandbox listeners accept their own tree's peers only
  int64_t uid_base = 0;                // first sandbox UID (0 = sandboxes keep the daemon's UID)
  int64_t uid_count = 4096;            // size of this daemon's UID range
  std::vector<std::string> protect;    // trees no sandbox may see (object store, ...)
  int64_t nproc = 1024;                // per-sandbox process cap (UID mode: RLIMIT_NPROC of its UID)
  int64_t mem_bytes = 0;               // RLIMIT_DATA of broker-backed (non-HIP) sandboxes (0 = none)
  double gang_grace_s = 10.0;          // after a gang rank fails, the others get this long before the gang is killed
  double fault_spawn_fail_rate = 0.0;  // fault injection: this share of pooled / warm-gang spawns dies in warm-up
  // the operator's RCCL / HSA environment for gang ranks (--gang-env K=V,...):
  // set unless the request's own env sets the key (a request may never set HSA_*)
  std::vector<std::pair<std::string, std::string>> gang_env;
  // gangs this daemon leads and keeps a warm rank set for (--gang-warm
  // "0,1,2,3;0,1"): each key is the HIP_VISIBLE_DEVICES list of a gang whose
  // first GPU is this daemon's; rank r of the set has its HIP context (and
  // torch's CUDA state) on device r before any request asks for it
  std::vector<std::string> gang_warm;
  // each GPU's slot CPUs (--gang-cpus): gang rank r runs on the CPUs of the
  // GPU it drives, not on this (the lead) daemon's -- the ranks' own threads,
  // RCCL's proxy threads and host staging then sit next to their GPU
  std::map<std::string, std::string> gang_cpus;
  // TCP a sandbox may connect() to ("open", "none", "egress:80,443"): its own
  // Landlock layer; gang ranks are always "open" (collective bootstrap)
  std::string sandbox_network = "open";
  int hbm_watchdog_ms = 100;           // VRAM scan period of running sandboxes (0 = off)
  int64_t hbm_slack = 256ll << 20;     // runtime overhead tolerated above a quota before the watchdog kills
  // admission, shared by every front-end replica attached to this daemon:
  // at most max_inflight admitted jobs, their HBM quotas within hbm_capacity;
  // the rest wait in arrival order (or get a 429 when they asked not to wait)
  int max_inflight = 0;                // 0 = unbounded
  int64_t hbm_capacity = 0;            // bytes; 0 = unbounded
  // this daemon's share of the node's host memory for sandbox trees: each
  // admitted job commits its trees' memory bound (sandbox_mem_bytes x ranks),
  // the commitments stay within it and the rest queue (0 = unbounded)
  int64_t mem_capacity = 0;
  double admit_timeout_s = 900.0;      // longest wait for admission (then 503)
  // standing commitments of the idle warm gang ranks placed on this GPU (the
  // front-end counts them per slot: one rank per warm gang size covering it)
  int64_t standing_hbm = 0;            // bytes of HBM they hold
  int64_t standing_mem = 0;            // bytes of host memory charged for them
  int64_t standing_rank_hbm = 0;       // one warm rank's share (a gang's rank runs as one)
  int64_t standing_rank_mem = 0;
  // per-sandbox containment, what the reference pod's container resources
  // bound (procmon.hpp): the whole process tree of a sandbox
  int64_t sandbox_mem_bytes = 0;       // anonymous + shmem memory (0 = off)
  int64_t sandbox_tasks = 0;           // processes + threads (0 = off)
  double sandbox_cpus = 0;             // CPU cores, throttled above (0 = off)
  int monitor_ms = 20;                 // monitor period (render-node holders' HBM, memory, tasks, CPU)
  std::string deny_ports;              // "p1,p2,...": TCP ports no sandbox may bind/connect (the service's listeners)
  // per-sandbox cgroup v2 leaves (cgroup2.hpp): auto | require | off | fake
  // (tests: a plain directory as the root); "" root = the daemon's own cgroup
  std::string cgroup_mode = "auto";
  std::string cgroup_root;
};


// kDirect: own HIP context, torch preloaded.  kLight: broker-backed, the CPU
// science stack preloaded.  kMin: broker-backed, only numpy + beekern
// preloaded -- forks ~5x faster (fork time scales with the zygote's RSS), for
// scripts that import nothing else.
// kMinCpu: a kMin sandbox whose broker session opens on first use
// (BEE_BROKER_LAZY=1), for scripts that import no GPU module: they never pay
// for a session.  Forked by the minimal zygotes.
// kNano: broker-backed, beekern only (numpy is imported on first use,
// ops/_lazy.py), for scripts whose imports are beekern + the standard
// library: numpy's ~90 mappings and ~7 MB of private memory are neither
// copied at the fork nor torn down at the exit.
// kNanoCpu: a kNano sandbox whose broker session opens on first use, for
// scripts that import the standard library only.
enum WorkerKind { kDirect = 0, kLight = 1, kMin = 2, kMinCpu = 3, kNano = 4, kNanoCpu = 5, kNumKinds = 6 };

enum class WorkerState { Spawning, Connected, Ready, Running, Exited, Failed };

struct Worker {
  // the running job's wake-up: its request thread waits on this (with the
  // pool's mutex) for "done" / exit, instead of on the pool-wide condition
  // every spawn, ready and exit of every sandbox notifies
  std::shared_ptr<std::condition_variable> job_cv;
  void notify_job() const {
    if (job_cv) job_cv->notify_all();
  }
  std::string id;
  std::string dir, ws, rp, meta;
  std::string gpus;
  pid_t pid = -1;
  int fd = -1;
  WorkerState state = WorkerState::Spawning;
  double t_spawn = 0, t_ready = 0, t_run = 0, t_exit = 0;  // CLOCK_MONOTONIC ms
  double warm_ms = 0;
  bool exited = false;
  int exit_code = 0;
  bool done = false;  // worker reported completion (outputs flushed) before exiting
  int done_code = 0;
  int final_code() const { return done ? done_code : exit_code; }
  int term_signal = 0;
  bool pooled = true;  // false: dedicated (gang / custom env) worker
  int kind = kDirect;
  int zygote = 0;  // index of the zygote that forked it
  int64_t hbm_quota = 0;
  // what the kernel broker charges this sandbox's connections against:
  // the quota (-1 once the sandbox is gone) and one account for all of them
  std::shared_ptr<std::atomic<int64_t>> quota_cell = std::make_shared<std::atomic<int64_t>>(0);
  std::shared_ptr<broker::Account> hbm = std::make_shared<broker::Account>();
  void set_quota(int64_t q) {
    hbm_quota = q;
    quota_cell->store(q);
  }
  std::string fail_reason;
  uid_t uid = 0;        // the sandbox's own UID (0 = runs as the daemon's user)
  pid_t peer_pid = 0;   // pid that connected as this worker (checked against the zygote's report)
  bool uid_released = false;
  int64_t hbm_killed = 0;  // VRAM seen when the watchdog killed it (0 = not killed)
  std::string kill_reason;  // why the monitor killed it (memory, processes, HBM)
  std::string cgroup;       // its cgroup v2 leaf while a job runs ("" = none)
  // monitor state (monitor thread only)
  bool has_render = false;  // holds a render-node descriptor: HBM checked every monitor tick
  double vram_next = 0;
  double cpu_last = -1, cpu_t_last = 0, cpu_debt = 0;
  bool throttled = false;
  std::string gang_key;  // member of this warm gang set ("" = none)
  bool gang_rank = false;  // a rank of a gang (its listeners take the other ranks' connections)
  bool died_warming = false;  // exited (or failed to spawn) before it became ready
};

class KernelBroker;

// A pre-imported Python process that forks sandboxes.  Zygote 0 preloads
// torch (direct sandboxes); light zygotes preload only the CPU stack, fork
// ~2x faster and run in parallel so refills keep up with the request rate.
struct Zygote {
  int index = 0;
  int kind = kDirect;
  pid_t pid = -1;
  int fd = -1;
  std::thread thread;
  std::mutex write_mu;
  std::atomic<bool> alive{false};
  // sandbox environment entries that are the same for every pooled spawn of
  // this zygote's kind: set once in the zygote's own environment, so a spawn
  // carries only what differs (or an "unset" for what it must not have)
  std::map<std::string, std::string> base_env;
};

struct ExecTimings {
  double acquire_ms = 0, stage_ms = 0, run_ms = 0, collect_ms = 0, total_ms = 0;
};

class SandboxPool {
 public:
  explicit SandboxPool(PoolConfig cfg);
  ~SandboxPool();
  bool start(std::string* err);
  void stop();

  // POST /v1/execute (pool mode). Returns response JSON; sets *http_status.
  Json execute(const Json& req, int* http_status);
  // POST /execute (pod mode, reference-compatible body {source_file, timeout}).
  Json execute_pod(const Json& req, int* http_status);

  Json status();
  std::string metrics_text();
  // gang support across front-end processes: stop admitting new jobs on this
  // GPU, wait until running ones drain; expires after ttl_s
  bool reserve(double ttl_s, double wait_s);
  void release();
  const PoolConfig& config() const { return cfg_; }
  bool healthy() const { return !zygotes_.empty() && zygotes_[0]->alive.load(); }
  // true if `pid` is a sandbox process (a zygote descendant, re-parented
  // escapees included) or runs under a sandbox UID: such peers are refused on
  // the executor's control socket
  bool is_sandbox_process(pid_t pid, uid_t uid);
  // the id of the running sandbox whose process tree holds a descriptor of
  // socket `inode` ("" = none): the front-ends' peer guard without UID mode
  std::string socket_holder(uint64_t inode);

 private:
  // zygote
  bool start_zygote(Zygote* z, std::string* err);
  void zygote_reader(Zygote* z);
  void send_zygote(Zygote* z, const Json& msg);
  Zygote* pick_zygote(int kind);
  bool any_zygote_alive() const;
  // workers
  void worker_acceptor();
  std::shared_ptr<Worker> spawn_worker(bool pooled, int kind, const std::string& gpus, const Json& extra_env,
                                       const std::string& fixed_ws = "", const std::string& fixed_rp = "",
                                       uid_t fixed_uid = 0, bool gang_rank = false, const std::string& fixed_id = "");
  // UID mode
  bool uid_mode() const { return uid_mode_; }
  uid_t alloc_uid_locked();
  void sweep_uid(uid_t uid, bool shm);  // SIGKILL every process of the UID (+ drop its /dev/shm files)
  void release_uid_locked(const std::shared_ptr<Worker>& w);
  void refill_locked();
  // warm gang sets (cfg_.gang_warm): spawn missing ones; take a ready one
  void refill_gangs_locked();
  std::vector<std::shared_ptr<Worker>> take_gang_locked(const std::string& key);
  // BEE_CPU_AFFINITY of gang rank r of a job on `gpus`: the CPUs of the slot
  // of the GPU it drives (cfg_.gang_cpus; "" = the lead daemon's own)
  std::string rank_cpus(const std::string& gpus, int r) const;
  std::map<std::string, std::vector<std::shared_ptr<Worker>>> gang_sets_;  // key -> ranks (spawning or ready)
  // consecutive warm-up failures of each key's set; at kGangWarmMaxFails the
  // key is no longer warmed (its gangs start cold) so a rank that cannot
  // initialise its device does not respawn a set of torch processes forever
  // and hold READY back for the whole start-up timeout
  std::map<std::string, int> gang_fails_;
  static constexpr int kGangWarmMaxFails = 3;
  bool fault_spawn_now() const;  // one draw of config.fault_spawn_fail_rate
  int target_of(int kind) const;
  std::shared_ptr<Worker> acquire(int kind, double timeout_s, std::string* err);
  broker::Peer peer_info(pid_t peer);
  bool wait_ready(const std::shared_ptr<Worker>& w, double timeout_s);
  void destroy(const std::shared_ptr<Worker>& w);
  void cleanup_loop();
  void recycle_idle();
  // out-of-process HBM enforcement: VRAM a sandbox's processes hold, from
  // the DRM fdinfo of their render-node descriptors (the in-process
  // interposer can be bypassed by the code it is meant to limit)
  // the containment monitor (procmon.hpp): memory, tasks, CPU and HBM of
  // every running sandbox's process tree
  void watchdog_loop();

  struct RunSpec {
    std::string script;
    std::vector<std::string> argv;
    double timeout_s = 60;
    int64_t hbm_quota = 0;
    Json env = Json::object();
    std::string code;  // the front-end's precompiled payload (opaque to the daemon), "" = none
    bool numpy_offload = false;  // the sandbox routes large numpy.random draws to the GPU (ops/numpy_offload.py)
    bool cow_trusted = false;    // the service's own job (self-warm): a learner's page set is trusted
  };
  struct RunResult {
    std::string stdout_text, stderr_text;
    int exit_code = 0;
    bool timed_out = false;
    bool died = false;  // worker vanished before running (spawn/warm failure)
  };
  RunResult run_in(const std::shared_ptr<Worker>& w, const RunSpec& spec);
  Json run_job(const Json& req, int* http_status, bool pod);

  PoolConfig cfg_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::shared_ptr<Worker>> workers_;  // by id
  std::map<pid_t, std::shared_ptr<Worker>> by_pid_;
  std::deque<std::shared_ptr<Worker>> ready_[kNumKinds];  // by WorkerKind
  int spawning_[kNumKinds] = {0, 0, 0, 0, 0, 0};
  std::unique_ptr<KernelBroker> broker_;
  // sandboxes' listening sockets accept only their own tree's peers
  // (listen_guard.hpp); null when off or unsupported (guard_why_ says why)
  std::unique_ptr<ListenGuard> listen_guard_;
  std::string guard_why_;
  // the listener guard's question: which sandbox (leader) does process `tgid`
  // belong to, and is it a gang rank (listen_guard.hpp)
  bool guard_resolve(pid_t tgid, pid_t* leader, bool* exempt);
  std::string broker_sock_path_;  // known before the broker starts (zygotes start first)
  bool want_broker_ = false;
  bool uid_mode_ = false;
  std::string isolation_note_;             // why UID mode is off (status / logs)
  Json net_layer_ = Json::object();        // what the zygotes' Landlock TCP layer applied (their hello)
  cg2::Manager cg_;                         // per-sandbox cgroup v2 leaves, when delegated
  std::vector<std::pair<std::string, int>> cleanup_leaves_;  // (leaf, tries) to remove (under mu_)
  std::string cg_why_;                      // why they are off
  std::atomic<int64_t> m_cg_leaves_{0}, m_cg_oom_kills_{0};
  // executed sandboxes' CPU: wait4 totals (zygote exit reports) and their own reports
  std::atomic<int64_t> m_sb_cpu_us_{0}, m_sb_minflt_{0}, m_sb_reaped_{0}, m_sb_wcpu_us_{0}, m_sb_wcpu_n_{0};
  std::vector<gid_t> dev_groups_;          // supplementary groups for GPU device nodes
  std::map<uid_t, int> uids_in_use_;       // UID -> live workers using it (gang ranks share one)
  std::deque<uid_t> uid_sweep_;            // released UIDs awaiting their sweep (cleanup thread)
  uint64_t next_uid_ = 0;
  bool light_ok_ = false;  // light sandboxes available (broker up, or a CPU-only pool)
  bool min_ok_ = false;    // minimal zygotes running
  bool nano_ok_ = false;   // nano (numpy-free) zygotes running
  // in-flight / HBM / host-memory bounds and the gang reservation, shared by
  // every front-end replica (admission.hpp); it publishes the load table
  std::unique_ptr<Admission> admission_;
  int inflight_spawns_ = 0;
  std::deque<std::pair<std::shared_ptr<Worker>, Json>> spawn_queue_;

  std::vector<std::unique_ptr<Zygote>> zygotes_;  // [0] = direct (torch), rest light
  std::atomic<uint64_t> rr_{0};
  std::atomic<bool> stopping_{false};
  int worker_listen_fd_ = -1;
  int wake_fd_ = -1;  // eventfd: a zygote reported a pid (parked hellos re-check)
  std::string worker_sock_path_;
  std::thread acceptor_thread_, cleanup_thread_, watchdog_thread_, refill_thread_;
  // pool refills run on their own thread: a request that takes a warm
  // sandbox only asks for its replacement (spawning one -- its directories,
  // its spawn line -- is ~0.1 ms of CPU that was on the request path)
  std::condition_variable refill_cv_;
  bool refill_wanted_ = false;
  void request_refill_locked() {
    refill_wanted_ = true;
    refill_cv_.notify_one();
  }
  void refill_loop();
  std::mutex cleanup_mu_;
  std::condition_variable cleanup_cv_;
  std::deque<std::string> cleanup_dirs_;
  std::mutex pod_mu_;  // pod mode: one execution at a time

  // metrics
  std::atomic<int64_t> m_exec_total_{0}, m_exec_failed_{0}, m_timeouts_{0}, m_spawned_{0}, m_spawn_failed_{0},
      m_recycled_{0}, m_gang_failfast_{0}, m_hbm_kills_{0}, m_mem_kills_{0}, m_task_kills_{0}, m_throttles_{0},
      m_gang_warm_hits_{0}, m_gang_cold_{0};
  std::atomic<int64_t> m_inflight_{0};
  double m_warm_ms_sum_ = 0, m_exec_ms_sum_ = 0, m_acquire_ms_sum_ = 0, m_fork_ms_sum_ = 0, m_worker_warm_ms_sum_ = 0;
  int64_t m_warm_count_ = 0, m_fork_count_ = 0;
};

}  // namespace bee
