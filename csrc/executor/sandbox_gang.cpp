// Sandbox pool: warm gang rank sets (multi-GPU jobs whose ranks already
// hold their devices) and the pools' targets per sandbox kind.
#include "sandbox_internal.hpp"

namespace bee {

using namespace sandbox_detail;

Json sandbox_detail::gang_rank_env(int r, int n, const std::vector<std::pair<std::string, std::string>>& gang_env) {
  Json e = Json::object();
  e.set("RANK", std::to_string(r));
  e.set("LOCAL_RANK", std::to_string(r));
  e.set("WORLD_SIZE", std::to_string(n));
  e.set("LOCAL_WORLD_SIZE", std::to_string(n));
  e.set("MASTER_ADDR", "127.0.0.1");
  // RCCL's bootstrap sockets: loopback only (a gang never leaves the node)
  e.set("NCCL_SOCKET_IFNAME", "lo");
  for (auto& kv : gang_env)
    if (!e.has(kv.first)) e.set(kv.first, kv.second);
  return e;
}

void SandboxPool::refill_gangs_locked() {
  // a gang's ranks fork from the torch zygote and initialise HIP on their own
  // device (BEE_DEVICE=r) plus torch's CUDA state, while nobody waits: a
  // gang request then starts its ranks like any pooled sandbox instead of
  // paying N forks + HIP + torch init on the request path
  if (cfg_.gang_warm.empty() || cfg_.pod_mode) return;
  for (const auto& key : cfg_.gang_warm) {
    auto it = gang_sets_.find(key);
    if (it != gang_sets_.end()) {
      bool broken = false, warm_failure = false, all_ready = true;
      for (auto& w : it->second) {
        broken = broken || w->exited || w->state == WorkerState::Failed;
        warm_failure = warm_failure || w->died_warming || w->state == WorkerState::Failed;
        all_ready = all_ready && w->state == WorkerState::Ready && !w->exited;
      }
      if (all_ready) gang_fails_[key] = 0;
      if (!broken) continue;
      if (warm_failure && ++gang_fails_[key] == kGangWarmMaxFails)
        BEE_WARN("warm gang set %s failed to start %d times: its gangs start cold from now on", key.c_str(),
                 kGangWarmMaxFails);
      for (auto& w : it->second) {  // one rank died while pooled: the set is useless
        if (w->pid > 0) kill(-w->pid, SIGKILL);
        release_uid_locked(w);
        workers_.erase(w->id);
        cleanup_dirs_.push_back(w->dir);
      }
      gang_sets_.erase(it);
    }
    if (gang_fails_[key] >= kGangWarmMaxFails) continue;
    const int n = 1 + (int)std::count(key.begin(), key.end(), ',');
    std::vector<std::shared_ptr<Worker>> set;
    std::string ws0, rp0;
    uid_t uid0 = 0;
    for (int r = 0; r < n; ++r) {
      Json e = gang_rank_env(r, n, cfg_.gang_env);
      if (fault_spawn_now()) e.set("BEE_FAULT_DIE_WARM", "1");
      if (cfg_.warm_gpu) {
        e.set("BEE_WARM_GPU", "1");
        e.set("BEE_WARM_TORCH", "1");
        e.set("BEE_DEVICE", std::to_string(r));
      }
      if (r > 0 && cfg_.jail) e.set("BEE_JAIL_SHARED", join_path(dirname_of(ws0), "tmp"));
      const std::string cpus = rank_cpus(key, r);
      if (!cpus.empty()) e.set("BEE_CPU_AFFINITY", cpus);
      auto w = spawn_worker(false, kDirect, key, e, ws0, rp0, uid0, true);
      w->gang_key = key;
      if (r == 0) {
        ws0 = w->ws;
        rp0 = w->rp;
        uid0 = w->uid;
      }
      set.push_back(w);
    }
    gang_sets_[key] = std::move(set);
  }
}

std::string SandboxPool::rank_cpus(const std::string& gpus, int r) const {
  auto it = cfg_.gang_cpus.find(nth_gpu(gpus, r));
  return it == cfg_.gang_cpus.end() ? std::string() : it->second;
}

std::vector<std::shared_ptr<Worker>> SandboxPool::take_gang_locked(const std::string& key) {
  auto it = gang_sets_.find(key);
  if (it == gang_sets_.end()) return {};
  for (auto& w : it->second)
    if (w->state != WorkerState::Ready || w->exited || w->fd < 0) return {};  // still warming (or broken: refill)
  auto set = std::move(it->second);
  gang_sets_.erase(it);
  for (auto& w : set) w->state = WorkerState::Running;
  request_refill_locked();
  return set;
}

bool SandboxPool::fault_spawn_now() const {
  return cfg_.fault_spawn_fail_rate > 0 &&
         (double)strtoul(random_hex(3).c_str(), nullptr, 16) / 16777216.0 < cfg_.fault_spawn_fail_rate;
}

int SandboxPool::target_of(int kind) const {
  // without a broker (CPU-only pools) the *_cpu kinds fold into their base
  // kind (handle(): mode "nano_cpu" -> kNano), so the base pool is sized for
  // both: a CPU-only node's stdlib scripts otherwise queue on the few warm
  // sandboxes of the GPU-script pool (hello on a CPU-only executor: p50
  // acquire 1.2 ms, 2755 vs 4531 RPS GPU-pinned, profiles/archive/r4_bench_suite.jsonl)
  if (kind == kLight) return light_ok_ ? cfg_.light_target : 0;
  if (kind == kMin)
    return light_ok_ && min_ok_ ? (!broker_ ? std::max(cfg_.min_target, cfg_.min_cpu_target) : cfg_.min_target) : 0;
  if (kind == kMinCpu) return broker_ && min_ok_ ? (cfg_.min_cpu_target >= 0 ? cfg_.min_cpu_target : cfg_.min_target) : 0;
  if (kind == kNano)
    return light_ok_ && nano_ok_ ? (!broker_ ? std::max(cfg_.nano_target, cfg_.nano_cpu_target) : cfg_.nano_target) : 0;
  if (kind == kNanoCpu)
    return broker_ && nano_ok_ ? (cfg_.nano_cpu_target >= 0 ? cfg_.nano_cpu_target : cfg_.nano_target) : 0;
  return cfg_.target;
}

}  // namespace bee
