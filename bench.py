"""Benchmark: aggregate agent-steps/s of the device-resident greedy rollout (BASELINE.json config 3).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Workload (per GPU, weak scaling): WarehouseMedium, 8 agents, B = 65,536 envs, greedy policy
(baseline/solvers.py:27-58) fused with Warehouse.step() (warehouse/core.py:262-442) and
auto-reset, philox draws keyed by global env id (rank r owns ids [r*B, (r+1)*B)).  One "step" = one
policy+transition for every env; every step writes rewards [B,8] f32 and dones [B] u8.  Ranks share
nothing on the data path (no RCCL); a gloo group only aligns the timing window and takes the max.

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  alt_launch_mode -- the same workload as a hipGraph of one-step launches (state through HBM)
  sampler_path -- the RLlib sampler route at the same B x NA: policy -> wh_vector_step (step +
                  auto-reset + float32 observation rows), with the observation kernel's roofline
                  (it writes B*NA*(9R+1)*4 bytes per step: HBM-write bound)
  policy_path  -- scripts/rollout.py's loop with the SAC policy network on the device
                  (wh_mlp_forward over all agent rows, then wh_vector_step), with the MLP kernel's
                  MFMA roofline (dense bf16 peak)
  roofline     -- algorithmic bytes of the step kernel / its mean duration (HIP events on the
                  launch stream), against the 8 TB/s HBM peak; `traffic` from the committed
                  rocprofv3 PMC summary (profiles/) when present.
  cpu_baseline -- the numpy restatement of warehouse.core.Warehouse.step() (oracle/core.py), one
                  env per process, step-only timing, on a bounded sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "rllib-warehouse_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "agent-steps/sec (aggregate) at B=65536 envs × 8 agents, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md, chip-level parameters (spec)
MFMA_BF16_PEAK_TFS = 2500.0   # dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md


def cpu_worker(args):
    """One process = one env (oracle restatement of warehouse.core.Warehouse.step()); returns
    (agent-steps, seconds spent inside step())."""
    variant, n, seconds, seed = args
    import numpy as np

    from oracle import core as oc

    np.random.seed(seed)
    env = oc.OracleWarehouse(variant, n)
    obs = env.reset()
    draws = env.draws
    steps, spent = 0, 0.0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS])
                         for i in range(n)])
        acts = oc.greedy(env.layout, flat, 0.0, draws)
        ad = {str(i): int(acts[i]) for i in range(n)}
        t0 = time.perf_counter()
        obs, _, dones, _ = env.step(ad)
        spent += time.perf_counter() - t0
        steps += 1
        if dones["__all__"]:
            obs = env.reset()
    return steps * n, spent


def cpu_baseline(variant, n, procs, seconds):
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(cpu_worker, [(variant, n, seconds, 1000 + i) for i in range(procs)])
    rate = sum(a / s for a, s in res if s > 0)
    return dict(value=rate, unit="agent-steps/s", cores=procs, kind="port",
                sample=f"{procs} processes x {seconds:.1f} s, 1 env each, {variant} N={n}, greedy actions, "
                       f"step-only time of oracle/core.py OracleWarehouse.step (numpy restatement of "
                       f"warehouse.core.Warehouse.step)")


def load_traffic(tag):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(tag, {}).get("bytes_per_launch")
    except Exception:
        return None


def config_name(variant, na, envs, policy):
    """BASELINE.json config this run corresponds to (SURVEY §8 notation), else 'custom'."""
    known = {("small", 4, 4096, "random"): "C2", ("medium", 8, 65536, "greedy"): "C3",
             ("large", 16, 65536, "greedy"): "C4"}
    return known.get((variant, na, envs, policy), "custom")


def load_issue(tag, steps_per_launch):
    """VALU issue view of the step kernel from the committed SQ counters (tools/profile_round.sh
    with SQ=1 -> profiles/pmc_traffic.json): per wave and env-step, VALU instructions and wave
    quad-cycles; one wave issues at most one VALU per quad-cycle (MI355X_MICROARCH.md)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        sq = json.load(open(path))[tag]["sq"]
        waves = sq["SQ_WAVES"]
        valu = sq["SQ_INSTS_VALU"] / waves / steps_per_launch
        cyc = sq["SQ_WAVE_CYCLES"] / waves / steps_per_launch
        return {"valu_per_wave_step": valu, "wave_quad_cycles_per_step": cyc, "valu_issue_frac": valu / cyc,
                "lds_per_wave_step": sq["SQ_INSTS_LDS"] / waves / steps_per_launch,
                "source": f"profiles/pmc_traffic.json:{tag}.sq"}
    except Exception:
        return None


def measure(env, mode, policy, K, W, chunk, dev, world, dist):
    """Time K steps of `mode`; returns (elapsed_s_max_over_ranks, kernel_ms, steps_per_launch)."""
    import torch

    B, NA = env.B, env.agent_slots
    stream = torch.cuda.current_stream(dev)
    if mode == "graph":
        rew = torch.zeros((1, B, NA), device=dev)
        dn = torch.zeros((1, B), dtype=torch.uint8, device=dev)

        def one():
            env.rollout(1, policy, 0.0, rewards=rew, dones=dn)

        for _ in range(max(W, 3)):
            one()
        torch.cuda.synchronize(dev)
        G = min(K, 200)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                one()
        torch.cuda.synchronize(dev)

        def run_steps(k):
            for _ in range(k // G):
                graph.replay()
            for _ in range(k % G):
                one()

        def timed_unit():
            graph.replay()
        per_unit_launches, spl = G, 1
    else:
        C = chunk
        rew = torch.zeros((C, B, NA), device=dev)
        dn = torch.zeros((C, B), dtype=torch.uint8, device=dev)

        def run_steps(k):
            while k > 0:
                c = min(C, k)
                env.rollout(c, policy, 0.0, rewards=rew[:c], dones=dn[:c])
                k -= c
        run_steps(max(W, 1))

        def timed_unit():
            env.rollout(C, policy, 0.0, rewards=rew, dones=dn)
        per_unit_launches, spl = 1, C

    # ---------------- timed region: barrier + sync on both sides, max over ranks
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(K)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---------------- kernel duration: HIP events on the launch stream around back-to-back
    # launches (a graph replay of G one-step launches, or one fused launch), median of 7
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
    for a, b in evs:
        a.record(stream)
        timed_unit()
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) / per_unit_launches for a, b in evs)
    return elapsed, kms[len(kms) // 2], spl


def measure_sampler(env, K, W, dev, world, dist):
    """The RLlib sampler route (scripts/train.py's workload): per step the device greedy policy
    stands in for the learner's policy, then wh_vector_step = step + auto-reset + observation
    rows [B,NA,9R+1] f32.  hipGraph of G steps.  Returns (elapsed_s, observe_kernel_ms)."""
    import torch

    stream = torch.cuda.current_stream(dev)

    def one():
        env.vector_step(env.policy("greedy", 0.0), autoreset=True, observe=True)

    for _ in range(max(W, 3)):
        one()
    torch.cuda.synchronize(dev)
    G = min(K, 100)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            one()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(K // G):
        graph.replay()
    for _ in range(K % G):
        one()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # observe kernel alone: 20 back-to-back launches between HIP events on the launch stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        for _ in range(20):
            env.observe()
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) / 20 for a, b in evs)
    return elapsed, kms[len(kms) // 2]


def measure_policy(env, K, W, dev, world, dist):
    """scripts/rollout.py's loop on the device: per step the SAC policy network
    (wh_mlp_forward, argmax) over all B x NA observation rows, then wh_vector_step (step +
    auto-reset + next rows).  hipGraph of G steps.  Returns (elapsed_s, mlp_kernel_ms, net)."""
    import torch

    import warehouse.policy as wp

    net = wp.MLPPolicy(env.variant, seed=7, device=dev)
    B, NA = env.B, env.agent_slots
    acts = torch.empty((B, NA), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    obs = env.observe()

    def one():
        net(obs.view(B * NA, -1), step=0, actions=acts.view(-1))
        env.vector_step(acts, autoreset=True, observe=True)

    for _ in range(max(min(W, 20), 3)):
        one()
    torch.cuda.synchronize(dev)
    G = min(K, 20)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            one()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(K // G):
        graph.replay()
    for _ in range(K % G):
        one()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        for _ in range(5):
            net(obs.view(B * NA, -1), step=0, actions=acts.view(-1))
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) / 5 for a, b in evs)
    return elapsed, kms[len(kms) // 2], net


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--variant", default="medium")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--policy", default="greedy", choices=["greedy", "random"])
    ap.add_argument("--mode", default="fused", choices=["graph", "fused"],
                    help="fused: --chunk steps per launch, state in registers (headline); "
                         "graph: hipGraph of one-step launches, state round-trips HBM every step")
    ap.add_argument("--chunk", type=int, default=200)
    ap.add_argument("--no-alt", action="store_true", help="skip the other launch mode")
    ap.add_argument("--no-sampler", action="store_true", help="skip the sampler-path (obs) measurement")
    ap.add_argument("--no-policy", action="store_true", help="skip the SAC-policy rollout measurement")
    ap.add_argument("--policy-steps", type=int, default=200)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = min(16, cpus)")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import warehouse

    B, NA, K, W = args.envs, args.agents, args.steps, args.warmup
    env = warehouse.BatchedWarehouse(args.variant, B, NA, seed=1234, env_offset=rank * B, device=dev)
    env.reset()
    words = env.layout.words_per_env
    out_b = 4 * NA + 1                       # rewards f32 x NA + done u8, per env-step

    elapsed, kernel_ms, spl = measure(env, args.mode, args.policy, K, W, args.chunk, dev, world, dist)
    value = world * B * NA * K / elapsed
    bytes_per_launch = B * (2 * 4 * words + spl * out_b)
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    alt = None
    if not args.no_alt:
        other = "graph" if args.mode == "fused" else "fused"
        el2, kms2, spl2 = measure(env, other, args.policy, K, W, args.chunk, dev, world, dist)
        bpl2 = B * (2 * 4 * words + spl2 * out_b)
        alt = {"mode": other, "value": world * B * NA * K / el2, "ms_per_step": el2 * 1e3 / K,
               "kernel_ms": kms2, "steps_per_launch": spl2, "bytes_per_launch": bpl2,
               "roofline_frac": bpl2 / (kms2 * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "traffic": load_traffic(f"{args.variant}_n{NA}_{other}")}

    sampler = None
    if not args.no_sampler:
        Ks = min(K, 1000)
        el3, oms = measure_sampler(env, Ks, W, dev, world, dist)
        obs_b = B * NA * env.obs_len * 4 + B * 4 * words     # rows written + packed state read
        sampler = {
            "workload": f"RLlib sampler route: device greedy actions -> wh_vector_step (step + auto-reset "
                        f"+ f32 observation rows [B,{NA},{env.obs_len}]), hipGraph of 100 steps",
            "value": world * B * NA * Ks / el3, "unit": "agent-steps/s", "steps": Ks,
            "ms_per_step": el3 * 1e3 / Ks,
            "roofline": {"bound": "hbm", "kernel": "k_observe", "kernel_ms": oms,
                         "bytes_per_launch": obs_b, "achieved": obs_b / (oms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": obs_b / (oms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": load_traffic(f"{args.variant}_n{NA}_observe")},
        }

    policy_line = None
    if not args.no_policy:
        Kp = min(K, args.policy_steps)
        el4, mms, net = measure_policy(env, Kp, W, dev, world, dist)
        rows = B * NA
        flop = 2.0 * rows * (net.in_dim * net.hidden[0] + net.hidden[0] * net.hidden[1] + net.hidden[1] * 9)
        policy_line = {
            "workload": f"scripts/rollout.py loop on device: SAC policy_model MLP [{net.in_dim},{net.hidden[0]},"
                        f"{net.hidden[1]},9] argmax over B*NA={rows} rows -> wh_vector_step (step + auto-reset + "
                        f"observation rows); random-init weights (no checkpoint ships with the reference)",
            "value": world * B * NA * Kp / el4, "unit": "agent-steps/s", "steps": Kp,
            "ms_per_step": el4 * 1e3 / Kp, "dtype": "bf16 MFMA, f32 accumulate",
            "roofline": {"bound": "mfma", "kernel": "k_mlp", "kernel_ms": mms, "flop_per_launch": flop,
                         "achieved": flop / (mms * 1e-3) / 1e12, "peak": MFMA_BF16_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": flop / (mms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFS,
                         "traffic": load_traffic(f"{args.variant}_n{NA}_mlp")},
        }

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/u32 packed integer state, f32 rewards",
            "data": "synthetic: philox-seeded episodes keyed by global env id, greedy policy on device",
            "config": {
                "workload": f"{config_name(args.variant, NA, B, args.policy)}: {args.variant} N={NA}, B={B} envs/GPU, "
                            f"{args.policy} policy fused with step + auto-reset (device-resident rollout)",
                "envs_per_gpu": B, "agents": NA, "variant": args.variant, "policy": args.policy,
                "launch": "hipGraph of 1-step launches" if args.mode == "graph" else f"{spl} steps per launch",
                "parallelism": f"independent env shards x{world}, no collectives",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic(f"{args.variant}_n{NA}_{args.mode}"),
                "kernel": f"k_step<Cfg<D,R,racks,{NA}>, {args.policy}>",
                "kernel_ms": kernel_ms,
                "steps_per_launch": spl,
                "bytes_per_launch": bytes_per_launch,
                "bytes_per_env_step": bytes_per_launch / B / spl,
                "issue": load_issue(f"{args.variant}_n{NA}_{args.mode}", spl),
                "note": "algorithmic bytes = 2 x packed state + per-step rewards/dones; the fused kernel "
                        "keeps state in registers and is VALU-issue bound (one wave per SIMD at B=65536): "
                        "`issue` is its VALU issue rate against one wave's ceiling (DESIGN.md §5)",
            },
            "alt_launch_mode": alt,
            "sampler_path": sampler,
            "policy_path": policy_line,
        }
        if not args.no_cpu_baseline and world == 1:   # reported at N=1 only
            procs = args.cpu_procs or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(args.variant, NA, procs, args.cpu_seconds)
            out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
