"""Service configuration: ``APP_*`` environment surface.

Parity with the reference `src/code_interpreter/config.py:18-80`, which uses
pydantic-settings with ``env_prefix="APP_"`` and ``env_ignore_empty=True``.
pydantic-settings is not available on the target image, so this is a small
typed loader with the same observable rules:

* each field ``foo_bar`` is read from ``APP_FOO_BAR`` (case-insensitive);
* empty values are ignored (the default stays);
* ``dict``/``list`` fields parse JSON, ``bytes`` fields take the raw UTF-8
  text (e.g. PEM contents), ``bool`` accepts 1/0/true/false/yes/no/on/off.

Fields below the ``# --- MI355X-native additions`` marker are new; they keep
the ``APP_`` prefix so a reference deployment's environment still works
unchanged.
"""

from __future__ import annotations

import copy
import dataclasses
import json
import os
import typing
from dataclasses import dataclass, field
from typing import Any, Dict, List, Mapping, Optional

ENV_PREFIX = "APP_"


def default_logging_config() -> Dict[str, Any]:
    # Same shape/format/levels as the reference (`config.py:22-47`) plus the
    # loggers this framework adds, so INFO from scheduler/executor is visible.
    return {
        "version": 1,
        "disable_existing_loggers": False,
        "handlers": {
            "console": {"class": "logging.StreamHandler", "formatter": "standard"},
        },
        "formatters": {
            "standard": {"format": "[%(levelname)s] [%(request_id)s] %(name)s: %(message)s"},
        },
        "root": {"level": "WARNING", "handlers": ["console"], "propagate": True},
        "loggers": {
            "kubectl": {"level": "INFO"},
            "grpc_server": {"level": "INFO"},
            "code_interpreter_servicer": {"level": "INFO"},
            "kubernetes_code_executor": {"level": "INFO"},
            "local_gpu_pool": {"level": "INFO"},
            "executor_client": {"level": "INFO"},
        },
    }


@dataclass
class Config:
    # logging config: https://docs.python.org/3/library/logging.config.html#logging-config-dictschema
    logging_config: Dict[str, Any] = field(default_factory=default_logging_config)
    # address:port of the gRPC server
    grpc_listen_addr: str = "0.0.0.0:50051"
    # address:port of the HTTP server
    http_listen_addr: str = "0.0.0.0:8000"
    # PEM text of the server certificate / key / CA (TLS only when all three are set)
    grpc_tls_cert: Optional[bytes] = None
    grpc_tls_cert_key: Optional[bytes] = None
    grpc_tls_ca_cert: Optional[bytes] = None
    # image for executor pods (kubernetes backend)
    executor_image: str = "localhost/bee-code-executor:local"
    # 'resources' of the executor container, e.g. {"limits": {"amd.com/gpu": 1}}
    executor_container_resources: Dict[str, Any] = field(default_factory=dict)
    # extra fields merged into the executor pod spec (runtimeClassName, volumes, ...)
    executor_pod_spec_extra: Dict[str, Any] = field(default_factory=dict)
    # directory of the file-object store
    file_storage_path: str = "./.tmp/files"
    # delete stored objects older than this many seconds (0 = keep forever,
    # the reference's behaviour)
    file_storage_ttl_seconds: float = 0.0
    # how many executor pods (kubernetes) to keep ready for immediate use
    executor_pod_queue_target_length: int = 5
    # prefix of executor pod names; 6 random [a-z0-9] follow
    executor_pod_name_prefix: str = "code-executor-"

    # --- MI355X-native additions -------------------------------------------
    # "local" = GPU-pinned sandbox pools on this node (default),
    # "kubernetes" = reference-style executor pods via kubectl.
    executor_backend: str = "local"
    # GPUs to pin executor pools to: None = autodetect, [] = CPU-only pool.
    gpu_ids: Optional[List[int]] = None
    # warm single-use "direct" sandboxes (own HIP context, for torch & co) per GPU
    workers_per_gpu_target: int = 2
    # warm single-use "light" sandboxes per GPU: no HIP context of their own,
    # beekern kernels run through the executor's kernel broker (cheap to refill)
    light_workers_per_gpu_target: int = 8
    # warm "minimal" sandboxes per GPU (numpy + beekern preloaded only: forks
    # ~5x faster than light ones; serves scripts importing nothing else)
    min_workers_per_gpu_target: int = 16
    # zygote processes forking minimal sandboxes per GPU
    min_zygotes_per_gpu: int = 4
    # warm minimal sandboxes per GPU for scripts that import no GPU module:
    # their kernel-broker session opens only if used (-1 = as many as the
    # minimal pool)
    min_cpu_workers_per_gpu_target: int = -1
    # warm "nano" sandboxes per GPU: beekern only, forked from zygotes that
    # never imported numpy (ops/_lazy.py), for scripts whose imports are
    # beekern + the standard library; 0 = such scripts use minimal sandboxes
    nano_workers_per_gpu_target: int = 16
    # zygote processes forking nano sandboxes per GPU
    nano_zygotes_per_gpu: int = 4
    # warm nano sandboxes per GPU for standard-library-only scripts (broker
    # session opened on first use; -1 = as many as the nano pool)
    nano_cpu_workers_per_gpu_target: int = -1
    # run the per-GPU kernel broker in the executor daemon
    broker_enabled: bool = True
    # zygote processes forking light sandboxes per GPU (fork parallelism)
    light_zygotes_per_gpu: int = 2
    # front-end (gRPC + HTTP) replica processes sharing the ports via
    # SO_REUSEPORT and the node's executors (0 = one per GPU, max 8)
    frontend_processes: int = 1
    # concurrent executions admitted per GPU pool (others queue)
    max_inflight_per_gpu: int = 16
    # per-sandbox HBM quota in bytes (0 = 288 GB / max_inflight_per_gpu minus reserve)
    hbm_quota_bytes: int = 0
    # HBM per GPU kept back from quotas (contexts, fragmentation)
    hbm_reserve_bytes: int = 16 * 1024**3
    # total HBM per GPU used for quota accounting (MI355X: 288 GB)
    hbm_total_bytes: int = 288 * 1000**3
    # seconds the service waits for every GPU's sandbox pools to reach target
    # before it reports ready (0 = do not wait)
    startup_warm_timeout_s: float = 300.0
    # Executes the supervisor drives through its own front-end replicas (per
    # GPU slot, 8 at a time per slot) before it reports ready: a freshly
    # started service is 15-25% slower per request for its first ~1-2k
    # Executes (the replicas' Python, the daemon's and broker's heaps, the
    # kernel's caches for the fork/exit path grow on first use); 0 = off
    startup_self_warm_executions: int = 3072
    # ... for at most this many seconds (a CPU-starved node stops early)
    startup_self_warm_max_s: float = 30.0
    # default execution timeout in seconds (reference: 60 s, `server.rs:201`)
    default_timeout: float = 60.0
    # where sandboxes (workspace + runtime-packages + logs) are created
    sandbox_root: str = "./.tmp/sandboxes"
    # path of the native executor daemon binary (None = in-tree build)
    executor_binary: Optional[str] = None
    # python interpreter used for sandbox zygotes
    worker_python: Optional[str] = None
    # initialise HIP + load the kernel library while a sandbox waits in the pool
    worker_warm_gpu: bool = True
    # report changed files recursively (reference: top level only, `server.rs:117-137`)
    changed_files_recursive: bool = False
    # local wheelhouse used for auto-installing missing imports (offline pip)
    wheelhouse: Optional[str] = None
    # fault injection: probability that spawning a sandbox fails (tests)
    fault_spawn_fail_rate: float = 0.0
    # recycle warm sandboxes that waited longer than this (seconds, 0 = never)
    worker_max_idle_s: float = 900.0
    # max bytes of stdout / stderr returned per execution
    max_output_bytes: int = 16 * 1024 * 1024
    # sandbox isolation (runtime/jail.py, csrc/jail): "auto" = on when the
    # native jail is built, "on" = required, "off" = none.  Landlock view of
    # the host (object store / other sandboxes / control sockets carved out),
    # signal + ptrace + abstract-socket scoping, seccomp, rlimits.
    sandbox_isolation: str = "auto"
    # first UID of the per-sandbox UID range (service running as root only;
    # 0 = sandboxes keep the service's UID).  Each GPU slot gets
    # sandbox_uid_count UIDs after it.  The reference ran executor pods as
    # UID 1001050000 (executor/Dockerfile:91-98).
    sandbox_uid_base: int = 1001050000
    sandbox_uid_count: int = 4096
    # pin each GPU slot's executor (and what it forks) and each front-end
    # replica to the CPUs of its GPU's NUMA node: "auto" (when the GPUs span
    # several NUMA nodes) or "off"
    numa_affinity: str = "auto"
    # with a CPU quota far below the CPUs the job may run on (cgroup cpu.max:
    # 16 CPUs of time on a 256-CPU host), pin the service to this many times
    # the quota's worth of CPUs, split between the GPU slots (0 = NUMA only).
    # 8: each slot's daemon, zygotes and sandboxes keep to their own CPUs.
    # Measured on MI355X with 8 slots folded onto one GPU and a 16-CPU quota
    # (bench.py --gpus 8 --fold, profiles/archive/r4_fold_rehearsal.md): 0 -> 2402 RPS
    # at 6.3 ms CPU per Execute, 2 -> 972 (4 CPUs a slot starve its zygotes),
    # 4 -> 1939, 8 -> 3416 RPS at 4.0 ms (the 1-slot run's 4.2); one slot:
    # 2x cut CPU 15-20% but not latency (profiles/archive/r3_cpu_quota_pinning_ab.log)
    cpu_quota_pin_factor: float = 8.0
    # the CPU quota the pinning assumes (0 = the cgroup's cpu.max): tests and
    # rehearsals on hosts without a quota
    cpu_quota_override: float = 0.0
    # a gang whose rank failed: seconds the other ranks get to finish before
    # the whole gang is killed (they are usually stuck in a collective)
    gang_failure_grace_s: float = 10.0
    # environment for every rank of a multi-GPU gang, set by the executor
    # under the request's own NCCL_* entries (operators may set HSA_* here,
    # requests may not).  A gang is one node's GPUs over xGMI: InfiniBand /
    # RoCE probing at communicator init is skipped.  Channel / protocol knobs
    # (NCCL_MIN_NCHANNELS, NCCL_PROTO, ...) are left to RCCL's gfx950 tuning
    # tables unless set here for a measured reason
    gang_rccl_env: Dict[str, str] = field(default_factory=lambda: {"NCCL_IB_DISABLE": "1"})
    # gang sizes kept warm on the node: for each size N, every aligned block
    # of N GPU slots (all 8; 0-3 and 4-7; the pairs) has a rank set whose
    # rank r already holds device r (HIP context + torch CUDA state) -- a
    # gang request takes it like a pooled sandbox instead of forking N ranks
    # and initialising HIP on the request path.  [] = every gang starts cold
    gang_warm_sizes: List[int] = field(default_factory=lambda: [2, 4, 8])
    # what one idle warm gang rank holds on its GPU (HIP context, torch's
    # CUDA state, loaded kernels) and in host memory: charged against the
    # slot's HBM and host-memory admission for every warm rank placed on it
    # (one per warm gang size: 3 x on an 8-GPU node), so 24 idle ranks per
    # node cannot overcommit either
    gang_warm_rank_hbm_bytes: int = 1 << 30
    gang_warm_rank_memory_bytes: int = 1 << 30
    # processes + threads per sandbox tree (the executor's monitor, any
    # mode; plus RLIMIT_NPROC of the sandbox UID in UID mode)
    sandbox_max_processes: int = 1024
    # private writable memory per sandbox process without a HIP runtime
    # (RLIMIT_DATA; 0 = unlimited): a runaway allocation is a MemoryError
    # in that sandbox, not node memory pressure for every GPU slot
    sandbox_memory_bytes: int = 64 * 1024**3
    # memory of a sandbox's whole process tree (anonymous + shmem; the
    # executor kills the sandbox above it).  limits.memory of
    # executor_container_resources overrides it (the reference pod's bound).
    # 0 = auto: the node's host-memory budget split over every admissible
    # sandbox (slots x max_inflight_per_gpu), within [2 GiB, 64 GiB]
    sandbox_tree_memory_bytes: int = 0
    # host memory the node's sandboxes may commit in all (their trees'
    # bounds, admitted like HBM: jobs queue when the next would exceed it).
    # 0 = auto: 85% of the smaller of MemTotal and the service's cgroup
    # memory limit; -1 = no aggregate bound
    host_memory_budget_bytes: int = 0
    # CPU cores per sandbox tree (0 = unbounded; throttled above): one
    # sandbox cannot take the whole node's CPU from the others.
    # limits.cpu of executor_container_resources overrides it
    sandbox_cpus: float = 8.0
    # period of the executor's containment monitor (ms): memory, processes,
    # CPU, and the HBM of sandboxes holding a render node
    sandbox_monitor_ms: int = 20
    # Landlock TCP layer on the zygotes (kernel ABI >= 4): sandboxes may not
    # bind or connect to the service's own gRPC / HTTP listeners (plus
    # sandbox_deny_ports); egress elsewhere stays open.  Off by default:
    # Landlock network rules allow single ports, so "all but these" is ~65k
    # rules, and every sandbox's own (nested) filesystem layer copies its
    # parent's rules -- measured +13 ms of CPU per sandbox.  Gang rendezvous
    # does not need it (FileStore in the gang's private directory).
    sandbox_net_layer: bool = False
    # what TCP a sandbox may connect() to, in its own Landlock layer (a few
    # rules, no measurable per-sandbox cost, tests/test_isolation_cpu.py):
    # "egress:80,443" (web egress only -- the service's gRPC / HTTP ports,
    # other sandboxes' servers and anything else on loopback are refused),
    # "egress:<ports>", "none", or "open" (the reference pod's network).
    # Default "open": Landlock rules name single ports, so an allow-list
    # cannot also keep a sandbox's loopback connections to its own servers on
    # ephemeral ports (torch.distributed's TCPStore of a one-rank job,
    # local test servers) -- measured, tests/test_sandbox_gpu.py
    # allreduce example.  Gang ranks always keep TCP (collective bootstrap);
    # kernels without Landlock ABI 4 leave it open.
    sandbox_network: str = "open"
    # a sandbox's listening sockets accept only connections from its own
    # process tree (and other hosts): its accept() calls go through the
    # executor daemon (seccomp user notifications, csrc/executor/listen_guard.hpp)
    # -- another sandbox cannot talk to its loopback servers, as with the
    # reference's pod per Execute.  Nothing on a request path that accepts
    # nothing; gang ranks are exempt (rank-to-rank bootstrap).
    sandbox_listen_guard: bool = True
    # UID mode (a root service with sandbox UIDs): the gRPC / HTTP front-ends
    # refuse calls whose peer socket belongs to a sandbox UID of this node
    # (one sock_diag lookup per call, nothing per sandbox;
    # services/peer_guard.py) -- the service's own API stays out of user
    # code's reach under the "open" network policy too
    api_refuse_sandbox_peers: bool = True
    sandbox_deny_ports: List[int] = field(default_factory=list)
    # per-sandbox cgroup v2 leaves (memory.max / pids.max / cpu.max,
    # cgroup.kill) beside the process-tree monitor: "auto" uses them when the
    # node delegates a cgroup v2 subtree to the service (else the monitor
    # alone, and the executor's status says why), "require" refuses to start
    # without one, "off" never.  sandbox_cgroup_root: the delegated directory
    # ("" = the executor's own cgroup)
    sandbox_cgroup: str = "auto"
    sandbox_cgroup_root: str = ""
    # numpy offload for every request (a request's numpy_offload field
    # overrides it): numpy.random draws of >= 2**20 elements live on the
    # sandbox's GPU and numpy functions on them run on the beekern kernels
    # (ops/numpy_offload.py); off = numpy semantics and placement unchanged
    numpy_offload: bool = False

    def __init__(self, _env: Optional[Mapping[str, str]] = None, **overrides: Any) -> None:
        env = os.environ if _env is None else _env
        lowered = {k.lower(): v for k, v in env.items() if k.upper().startswith(ENV_PREFIX)}
        hints = typing.get_type_hints(type(self))
        for f in dataclasses.fields(self):
            if f.name in overrides:
                value = overrides.pop(f.name)
            else:
                raw = lowered.get((ENV_PREFIX + f.name).lower())
                if raw is not None and raw != "":
                    value = _coerce(f.name, raw, hints[f.name])
                elif f.default is not dataclasses.MISSING:
                    value = copy.deepcopy(f.default)
                else:
                    value = f.default_factory()  # type: ignore[misc]
            setattr(self, f.name, value)
        if overrides:
            raise TypeError(f"unknown config fields: {sorted(overrides)}")

    def as_dict(self) -> Dict[str, Any]:
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}


_TRUE = {"1", "true", "yes", "on", "y", "t"}
_FALSE = {"0", "false", "no", "off", "n", "f"}


def _coerce(name: str, raw: str, hint: Any) -> Any:
    origin = typing.get_origin(hint)
    args = typing.get_args(hint)
    if origin is typing.Union:  # Optional[X]
        inner = [a for a in args if a is not type(None)]
        if raw.strip().lower() in ("null", "none"):
            return None
        return _coerce(name, raw, inner[0])
    try:
        if hint is bytes:
            return raw.encode("utf-8")
        if hint is str:
            return raw
        if hint is bool:
            low = raw.strip().lower()
            if low in _TRUE:
                return True
            if low in _FALSE:
                return False
            raise ValueError(raw)
        if hint is int:
            return int(raw.strip())
        if hint is float:
            return float(raw.strip())
        if origin in (dict, list) or hint in (dict, list):
            value = json.loads(raw)
            expected = origin or hint
            if not isinstance(value, expected):
                raise ValueError(f"expected JSON {expected.__name__}")
            if origin is list and args and args[0] is int:
                value = [int(v) for v in value]
            return value
    except (ValueError, json.JSONDecodeError) as e:
        raise ValueError(f"invalid value for {ENV_PREFIX}{name.upper()}: {raw!r} ({e})") from e
    raise TypeError(f"unsupported config type for {name}: {hint!r}")
