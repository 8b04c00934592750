# Sandboxes that import torch get a direct (HIP-initialised) worker pinned to
# the request's GPU(s); HIP_VISIBLE_DEVICES is already set.
import torch

x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
y = x @ x.T
torch.cuda.synchronize()
print(torch.cuda.get_device_name(0), float(y.float().abs().mean()))
