"""The sampler route one launch pair at a time (BatchedWarehouse.sampler_step) against the two-stream
SamplerPipeline (the rows of step s on a side stream while step s + 1 runs), each as hipGraph
replays of 100 steps.

    python tools/pipeline_probe.py [--variant large --agents 16 --replays 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402
from warehouse.vector import SamplerPipeline  # noqa: E402


def timed(graph, replays, dev):
    graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(replays):
        graph.replay()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / replays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="large")
    ap.add_argument("--agents", type=int, default=16)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--replays", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    G = 100
    env = warehouse.BatchedWarehouse(a.variant, a.envs, a.agents, seed=3, device=dev)
    env.reset()
    for _ in range(3):
        env.sampler_step("greedy", 0.0)
    torch.cuda.synchronize(dev)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        for _ in range(G):
            env.sampler_step("greedy", 0.0)
    pipe = SamplerPipeline(env, "greedy", 0.0)
    pipe.begin()
    for _ in range(4):
        pipe.step()
    pipe.end()
    torch.cuda.synchronize(dev)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        pipe.begin()
        for _ in range(G):
            pipe.step()
        pipe.end()
    for r in range(a.replays):
        us1 = timed(g1, 1, dev) / G * 1e6
        us2 = timed(g2, 1, dev) / G * 1e6
        print(f"{a.variant}-{a.agents} B={a.envs} round {r}: sampler_step {us1:.2f} us/step, "
              f"SamplerPipeline {us2:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
