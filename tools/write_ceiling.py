"""Achievable HBM write rate for buffers the size of the observation rows (torch fill_ = a plain
streaming-store kernel): the practical ceiling k_observe / k_sampler are compared against.

Two views per size: the same buffer rewritten (what a 1-step sampler route does every step: the
buffer may stay partly resident in the 256 MB MALL), and a ring of distinct chunks of that size
covering 3.4 GB (what a 20-step rollout fragment writes: every chunk is new memory, so the stores
stream to HBM).
    python tools/write_ceiling.py
"""
import torch

RING_BYTES = 3.44e9
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
    del x
    k = max(2, int(RING_BYTES / (n * 4)))
    ring = torch.empty((k, n), device="cuda")
    for i in range(k):
        ring[i].fill_(1.0)
    torch.cuda.synchronize()
    a.record()
    for i in range(k):
        ring[i].fill_(2.0)
    b.record()
    torch.cuda.synchronize()
    us_ring = a.elapsed_time(b) / k * 1e3
    del ring
    print(f"fill {mb:7.1f} MB  same buffer {us:8.1f} us {n * 4 / us / 1e3:7.1f} GB/s   ring of {k} x {mb:.1f} MB "
          f"{us_ring:8.1f} us {n * 4 / us_ring / 1e3:7.1f} GB/s", flush=True)
