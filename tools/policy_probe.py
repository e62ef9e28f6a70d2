"""The policy route of bench.py's policy leg alone (scripts/rollout.py's loop on the device: bf16 SAC
network on the fragment operand -> wh_vector_step_x), as a hipGraph of 20 steps replayed R times;
prints us per step.  WH_SAMPLER_UNFUSED=1 (A/B): the step and the operand in two launches."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402
import warehouse.policy as wp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="medium")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--replays", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    env = warehouse.BatchedWarehouse(a.variant, a.envs, a.agents, seed=3, device=dev)
    env.reset()
    net = wp.MLPPolicy(env.variant, seed=7, device=dev)
    B, NA = env.B, env.agent_slots
    acts = torch.empty((B, NA), dtype=torch.int32, device=dev)
    obs = env.observe_x()

    def one():
        net.forward_x(obs, B * NA, step=0, actions=acts.view(-1))
        env.vector_step_x(acts, autoreset=True)

    for _ in range(5):
        one()
    torch.cuda.synchronize(dev)
    G = 20
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            one()
    graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.replays):
        graph.replay()
    torch.cuda.synchronize(dev)
    us = (time.perf_counter() - t0) / (a.replays * G) * 1e6
    print(f"{a.variant}-{a.agents} B={a.envs}: policy route {us:.1f} us per step, {B * NA / us * 1e6:.3e} agent rows/s",
          flush=True)


if __name__ == "__main__":
    main()
