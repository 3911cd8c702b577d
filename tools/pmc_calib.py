"""Known-byte-count kernels for calibrating rocprofv3 PMC counters:
a 1 GiB fp32 sum (reads 1 GiB) and a 1 GiB copy (reads 1 GiB, writes 1 GiB)."""
import torch

n = 1 << 28
x = torch.ones(n, device="cuda")
y = torch.empty_like(x)
torch.cuda.synchronize()
for _ in range(3):
    s = x.sum()
    y.copy_(x)
torch.cuda.synchronize()
print("sum", float(s))
