"""Which hipBLASLt kernel does torch pick for the bf16 GEMMs beekern is
compared against?  Run under `rocprofv3 --kernel-trace --stats`; the kernel
names (and the code object they come from) go into the stats CSV.

    rocprofv3 --kernel-trace --stats -d gpurun_out/blaslt -- python tools/probe/blaslt_kernel_probe.py
"""

import torch

for n in (4096, 8192):
    a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    bt = torch.empty(n, n, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    for out_dtype in (torch.bfloat16,):
        for _ in range(5):
            c = a @ bt.T
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        c = a @ bt.T
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 10
    print(f"{n}^3 TN bf16: {ms * 1e3:.0f} us  {2 * n**3 / ms / 1e9:.0f} TFLOP/s", flush=True)
