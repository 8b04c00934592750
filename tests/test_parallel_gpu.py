"""RCCL on the GPU box: the native all-reduce sweep at every power-of-two
GPU count the box shows (1 on the per-round box; 2/4/8 on a full node), in
f32 and bf16, correctness-checked by the tool, with a bus-bandwidth floor
for multi-GPU counts."""

import pytest

pytestmark = pytest.mark.gpu


def _counts():
    import torch

    n = torch.cuda.device_count()
    return [c for c in (1, 2, 4, 8) if c <= n] or [1]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_native_rccl_allreduce_sweep(dtype):
    from bee_code_interpreter_fs_amd.parallel import busbw_budget_gbps, rccl_allreduce_sweep

    for n in _counts():
        recs = rccl_allreduce_sweep(gpus=n, min_bytes="4K", max_bytes="256M", iters=5, dtype=dtype)
        head, rows = recs[0], recs[1:]
        assert head["gpus"] == n and head["dtype"] == dtype
        assert rows and all(r["checked"] for r in rows), rows
        assert rows[-1]["bytes"] == 256 << 20
        small = rows[0]  # 4 KiB: the latency end of the sweep
        assert small["bytes"] == 4096 and small["us"] > 0, small
        if n > 1:
            # xGMI: at 256 MB a real fraction of the gang's link budget ((n-1)
            # links of ~153 GB/s; 7 at n = 8), and nothing beyond it
            assert 0.25 * busbw_budget_gbps(n) < rows[-1]["busbw_GBps"] < busbw_budget_gbps(n) * 1.05, rows[-1]
