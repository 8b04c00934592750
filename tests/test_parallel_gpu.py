"""RCCL on the GPU box: native all-reduce sweep + a gang sandbox job."""

import pytest

pytestmark = pytest.mark.gpu


def test_native_rccl_allreduce_sweep():
    from bee_code_interpreter_fs_amd.parallel import rccl_allreduce_sweep

    recs = rccl_allreduce_sweep(min_bytes="4K", max_bytes="64M", iters=5)
    head, rows = recs[0], recs[1:]
    assert head["gpus"] >= 1
    assert rows and all(r["checked"] for r in rows)
    assert rows[-1]["bytes"] == 64 << 20
