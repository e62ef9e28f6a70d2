"""wh_vector_step (external actions, auto-reset, f32 rows) at Medium-8, B = 65,536, three forms of
the same ascending-order step, each as 5 replays of a 100-step hipGraph: the fast instance (no mask,
no order -- RLlib's common case), the generic instance (an all-true mask) and the dict-order instance
(every env's dict in ascending order, given explicitly as `order`).

    python tools/vector_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, NA, G = 65536, 8, 100
    env = warehouse.BatchedWarehouse("medium", B, NA, seed=3, device=dev)
    env.reset()
    acts = torch.randint(0, 9, (B, NA), device=dev, dtype=torch.int32)
    mask = torch.ones(B, dtype=torch.bool, device=dev)
    order = torch.arange(NA, device=dev, dtype=torch.int32).repeat(B, 1).contiguous()
    forms = {"fast (no mask, no order)": dict(), "generic (all-true mask)": dict(mask=mask),
             "dict order (ascending, explicit)": dict(order=order),
             "fast, step only (no rows)": dict(observe=False),
             "generic, step only (no rows)": dict(mask=mask, observe=False),
             "dict order, step only (no rows)": dict(order=order, observe=False)}
    graphs = {}
    for name, kw in forms.items():
        for _ in range(3):
            env.vector_step(acts, **kw)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(G):
                env.vector_step(acts, **kw)
        graphs[name] = g
    for r in range(3):
        for name, g in graphs.items():
            g.replay()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize(dev)
            us = (time.perf_counter() - t0) / (5 * G) * 1e6
            print(f"round {r} {name:34s} {us:7.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
