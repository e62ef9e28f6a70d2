"""The sampler route alone, for a kernel trace of its graph replays (bench.py's sampler_path leg):
BatchedWarehouse.sampler_step (device greedy fused into a 1-step launch, then wh_observe's f32 rows)
captured as a hipGraph of 100 steps and replayed R times; prints the per-step wall time.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sampler -o run -- python3 tools/sampler_probe.py
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="medium")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--replays", type=int, default=5)
    ap.add_argument("--fragment", type=int, default=0,
                    help="K > 0: also time wh_sampler_rollout launches of K steps (rollout fragments)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    env = warehouse.BatchedWarehouse(a.variant, a.envs, a.agents, seed=3, device=dev)
    env.reset()
    for _ in range(5):
        env.sampler_step("greedy", 0.0, observe=True)
    torch.cuda.synchronize(dev)
    G = 100
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            env.sampler_step("greedy", 0.0, observe=True)
    torch.cuda.synchronize(dev)
    graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.replays):
        graph.replay()
    torch.cuda.synchronize(dev)
    us = (time.perf_counter() - t0) / (a.replays * G) * 1e6
    print(f"{a.variant}-{a.agents} B={a.envs}: sampler step {us:.2f} us, "
          f"{a.envs * a.agents / us * 1e6:.3e} agent-steps/s", flush=True)
    if a.fragment:
        K = a.fragment
        obs = torch.empty((K, a.envs, env.agent_slots, env.obs_len), device=dev)
        rew = torch.empty((K, a.envs, env.agent_slots), device=dev)
        dn = torch.empty((K, a.envs), dtype=torch.uint8, device=dev)
        for _ in range(3):
            env.sampler_rollout(K, "greedy", 0.0, obs=obs, rewards=rew, dones=dn)
        s = torch.cuda.current_stream(dev)
        times = []
        for _ in range(a.replays):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            env.sampler_rollout(K, "greedy", 0.0, obs=obs, rewards=rew, dones=dn)
            e1.record(s)
            torch.cuda.synchronize(dev)
            times.append(e0.elapsed_time(e1) * 1e3)
        us = sorted(times)[len(times) // 2] / K
        print(f"{a.variant}-{a.agents} B={a.envs}: sampler rollout of {K} steps per launch: {us:.2f} us per step, "
              f"{a.envs * a.agents / us * 1e6:.3e} agent-steps/s (launches {', '.join(f'{t:.0f}' for t in times)} us)",
              flush=True)


if __name__ == "__main__":
    main()
