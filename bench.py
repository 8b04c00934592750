"""Headline benchmark: Execute RPCs/sec + p50 latency of the benchmark-numpy
payload on N GPU-pinned executor pods (BASELINE.json metric / configs 3-4).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W

Topology: rank 0 hosts the service (gRPC front-end + scheduler + one native
bee-executor per GPU, each with a warm pool of single-use sandboxes pinned to
its MI355X).  Every rank runs ``--concurrency`` closed-loop gRPC clients
against it, so offered load grows with N (weak scaling).  One "step" = every
client completes one Execute RPC of the payload (examples/benchmark_numpy_gpu.py:
1e8 f64 Philox rand + fused square-sum + 4096^3 bf16 MFMA GEMM, all on the
sandbox's GPU, result printed and verified).  K steps are timed between a
barrier + torch.cuda.synchronize() on every rank; the time is the max over
ranks; ``value`` = total completed RPCs / that time.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PAYLOAD = os.path.join(ROOT, "examples", "benchmark_numpy_gpu.py")
EXPECTED = 10**8 / 3  # E[sum U^2]


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--concurrency", type=int, default=4, help="closed-loop clients per GPU")
    p.add_argument("--pool-target", type=int, default=8, help="warm sandboxes per GPU")
    p.add_argument("--payload", default=PAYLOAD)
    p.add_argument("--no-gang-check", action="store_true")
    return p.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def percentile(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    k = max(0, min(len(xs) - 1, int(round(q / 100.0 * (len(xs) - 1)))))
    return xs[k]


async def client_loop(stub, pb, source, n, lat, errors, exec_times, phases):
    for _ in range(n):
        t = time.perf_counter()
        try:
            r = await stub.Execute(pb.ExecuteRequest(source_code=source), timeout=600)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e)[:300])
            continue
        lat.append((time.perf_counter() - t) * 1e3)
        for k, v in r.timings_ms.items():
            phases.setdefault(k, []).append(v)
        ok = r.exit_code == 0 and "Result:" in r.stdout
        if ok:
            try:
                val = float(r.stdout.split("Result:")[1].split()[0])
                ok = abs(val - EXPECTED) < 5e4
                exec_times.append(float(r.stdout.split("Execution Time:")[1].split()[0]) * 1e3)
            except (IndexError, ValueError):
                ok = False
        if not ok:
            errors.append(f"exit={r.exit_code} stdout={r.stdout[-200:]!r} stderr={r.stderr[-500:]!r}")


async def run_clients(target, source, concurrency, n):
    import grpc

    from bee_code_interpreter_fs_amd.models import proto as pb

    lat, errors, exec_times, phases = [], [], [], {}
    async with grpc.aio.insecure_channel(target) as ch:
        stub = pb.CodeInterpreterServiceStub(ch)
        await asyncio.gather(
            *(client_loop(stub, pb, source, n, lat, errors, exec_times, phases) for _ in range(concurrency))
        )
    return lat, errors, exec_times, phases


def main():
    args = parse_args()
    world, rank, local = dist_env()
    n_gpus = args.gpus if world == 1 else world
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
    torch.cuda.set_device(local)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    source = open(args.payload).read()
    loop = asyncio.new_event_loop()
    service = None
    tmp = tempfile.mkdtemp(prefix="bee-bench-", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    port = [None]
    if rank == 0:
        from tests.harness import ServiceHarness  # full service in a background thread

        service = ServiceHarness(
            tmp,
            gpu_ids=list(range(n_gpus)),
            workers_per_gpu_target=1,  # direct (own HIP context) sandboxes: the payload does not need them
            light_workers_per_gpu_target=args.pool_target,
            max_inflight_per_gpu=max(args.concurrency * 2, 4),
            default_timeout=300.0,
        )
        service.start()
        port = [service.grpc_port]
    if world > 1:
        dist.broadcast_object_list(port, src=0)
    target = f"127.0.0.1:{port[0]}"

    # warm-up rounds (also pages in every pool)
    loop.run_until_complete(run_clients(target, source, args.concurrency, args.warmup))
    barrier()
    t0 = time.perf_counter()
    lat, errors, exec_times, phases = loop.run_until_complete(run_clients(target, source, args.concurrency, args.steps))
    barrier()
    elapsed = time.perf_counter() - t0

    gathered = [(elapsed, lat, errors, exec_times, phases)]
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, (elapsed, lat, errors, exec_times, phases))
    max_elapsed = max(g[0] for g in gathered)
    all_lat = [x for g in gathered for x in g[1]]
    all_err = [x for g in gathered for x in g[2]]
    all_exec = [x for g in gathered for x in g[3]]
    all_phases = {}
    for g in gathered:
        for k, v in g[4].items():
            all_phases.setdefault(k, []).extend(v)

    gang = None
    if rank == 0 and n_gpus > 1 and not args.no_gang_check:
        gang = gang_allreduce_check(service, n_gpus)

    if rank == 0:
        total = len(all_lat)
        rps = total / max_elapsed if max_elapsed > 0 else 0.0
        out = {
            "metric": "Execute RPCs/sec (benchmark-numpy payload via HIP kernels)",
            "value": round(rps, 3),
            "unit": "requests/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_elapsed * 1e3 / max(args.steps, 1), 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "float64 (rand/square/sum) + bf16 (GEMM)",
            "data": "synthetic (device Philox RNG; random bf16 GEMM operands)",
            "config": {
                "model": "benchmark-numpy.py payload: 1e8 f64 rand+square+sum + 4096^3 bf16 GEMM per Execute",
                "global_batch": args.concurrency * world,
                "seq_len": None,
                "parallelism": f"{n_gpus} GPU-pinned executor pods, {args.concurrency * world} concurrent clients",
            },
            "p50_latency_ms": round(statistics.median(all_lat), 3) if all_lat else None,
            "p95_latency_ms": round(percentile(all_lat, 95), 3) if all_lat else None,
            "p50_in_sandbox_exec_ms": round(statistics.median(all_exec), 3) if all_exec else None,
            "p50_phase_ms": {k: round(statistics.median(v), 3) for k, v in sorted(all_phases.items())},
            "completed": total,
            "errors": len(all_err),
        }
        if all_err:
            out["first_error"] = all_err[0][:400]
        if gang is not None:
            out["gang_allreduce"] = gang
        try:
            st = service.call(service.ctx.code_executor.status(), timeout=30)
            keys = ("mean_warm_ms", "mean_worker_warm_ms", "mean_fork_ms", "mean_acquire_ms", "executions")
            out["executors"] = [{k: round(s["executor"].get(k, 0), 3) for k in keys} for s in st["slots"]]
        except Exception as e:  # noqa: BLE001
            out["executors"] = repr(e)[:200]
        print(json.dumps(out), flush=True)
        service.stop()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    loop.close()


GANG_SCRIPT = """
import os, time, torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
dist.init_process_group("nccl", rank=rank, world_size=world)
x = torch.full((64 << 20,), float(rank + 1), device="cuda")  # 256 MB f32
dist.all_reduce(x); torch.cuda.synchronize()
t = time.perf_counter(); iters = 10
for _ in range(iters):
    dist.all_reduce(x)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / iters
ok = bool(torch.allclose(x[:16], torch.full((16,), world * (world + 1) / 2 * world ** (iters + 1) / world, device="cuda"), rtol=1e-3))
busbw = 2 * (world - 1) / world * x.numel() * 4 / dt / 1e9
if rank == 0:
    print(f"allreduce_ok={ok} busbw_GBps={busbw:.1f}")
dist.destroy_process_group()
"""


def gang_allreduce_check(service, n):
    """BASELINE config 5: an 8-GPU torch.distributed (RCCL) job inside one
    gang sandbox, dispatched through the service like any other request."""
    try:
        r = service.call(
            service.ctx.code_executor.execute(source_code=GANG_SCRIPT, gpus=n, nprocs=n, timeout=240), timeout=300
        )
        line = [l for l in r.stdout.splitlines() if l.startswith("allreduce_ok")]
        return {"exit_code": r.exit_code, "result": line[0] if line else None, "stderr_tail": r.stderr[-300:] if r.exit_code else ""}
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)[:300]}


if __name__ == "__main__":
    main()
