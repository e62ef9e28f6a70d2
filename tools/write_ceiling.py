"""Achievable HBM write rate for buffers the size of the observation rows (torch fill_ = a plain
streaming-store kernel): the practical ceiling k_observe is compared against."""
import torch

for mb in (38.8, 172.0, 608.2, 1200.0):
    n = int(mb * 1e6 / 4)
    x = torch.empty(n, device="cuda")
    for _ in range(3):
        x.fill_(1.0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        x.fill_(2.0)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    print(f"fill {mb:7.1f} MB  {us:8.1f} us  {n * 4 / us / 1e3:7.1f} GB/s", flush=True)
