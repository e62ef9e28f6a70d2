"""Benchmark: aggregate agent-steps/s of the device-resident greedy rollout (BASELINE.json config 3).

    python bench.py [--gpus N --steps K --warmup W]      (N > 1: starts the N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Without a launcher, --gpus N > 1 makes this process start N child processes with
torch.distributed.run's environment (launch_ranks; the parent touches no GPU); under a launcher,
WORLD_SIZE must equal --gpus.  More ranks than cards is refused unless --rehearse-shared-devices
(then the line's metric says REHEARSAL and `devices` records the sharing).

Workload (per GPU, weak scaling): WarehouseMedium, 8 agents, B = 65,536 envs, greedy policy
(baseline/solvers.py:27-58) fused with Warehouse.step() (warehouse/core.py:262-442) and
auto-reset, philox draws keyed by global env id (rank r owns ids [r*B, (r+1)*B)).  One "step" = one
policy+transition for every env; every step writes rewards [B,8] f32 and dones [B] u8.  Ranks share
nothing on the data path (no RCCL); a gloo group only aligns the timing window and takes the max.

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  alt_launch_mode -- the same workload as a hipGraph of one-step launches (state through HBM)
  desync_episodes -- the headline launches after desynchronising the episodes (every step some
                  envs of each wave end and reset), with its kernel time relative to the headline
  sampler_path -- the RLlib sampler route at the same B x NA: policy -> wh_vector_step (step +
                  auto-reset + float32 observation rows), with the observation kernel's roofline
                  (it writes B*NA*(9R+1)*4 bytes per step: HBM-write bound)
  policy_path  -- scripts/rollout.py's loop with the SAC policy network on the device
                  (wh_mlp_forward over all agent rows, then wh_vector_step), with the MLP kernel's
                  MFMA roofline (dense bf16 peak); policy_path_f32 the same with the exact-f32
                  network (f32 MFMA peak)
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
MFMA_F32_PEAK_TFS = 157.3     # f32-input MFMA peak (= the f32 vector rate), MI355X_MICROARCH.md
# VALU issue peak of the chip: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 2 cycles
# at the 2.4 GHz max clock (MI355X_MICROARCH.md, execution model: a wave issues each VALU over 2
# cycles; one wave ALONE sustains one per 4, so a one-wave-per-SIMD kernel tops out at half of this)
SIMDS = 256 * 4
VALU_PEAK_GIPS = SIMDS * 2.4 / 2   # G wave-instructions/s


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


def host_cores():
    """Host cores this job may use: os.cpu_count(), narrowed by the CPU affinity mask and by a
    cgroup v2 CPU quota (a GPU box shares a large host, so os.cpu_count() alone over-counts).
    Returns (cores, detail)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    cores = min(c for c in (total, aff, quota) if c)
    return cores, f"os.cpu_count()={total}, affinity={aff}, cgroup quota={quota or 'none'}"


def cpu_baseline(variant, n, procs, seconds, detail=""):
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    # close + join, not the context manager: Pool.__exit__ terminates the workers with SIGTERM, which a
    # profiler's signal handler logs as an abort per worker (noise in every fault scan of the log)
    pool = ctx.Pool(procs)
    try:
        res = pool.map(cpu_worker, [(variant, n, seconds, 1000 + i) for i in range(procs)])
    finally:
        pool.close()
        pool.join()
    rate = sum(a / s for a, s in res if s > 0)
    return dict(value=rate, unit="agent-steps/s", cores=procs, kind="port",
                sample=f"one process per host core ({procs}; {detail}) x {seconds:.1f} s, 1 env each, "
                       f"{variant} N={n}, greedy actions, step-only time of oracle/core.py "
                       f"OracleWarehouse.step (numpy restatement of warehouse.core.Warehouse.step)")


def source_sha():
    """The tree's source sha (warehouse/_native.py:tree_source_sha: csrc/*.hip, *.h, *.cpp, the
    Makefile and include/warehouse_amd.h -- the hash the Makefile bakes into wh_version()):
    profile-derived fields are reported only when the committed profile was taken from the same
    sources, and the run refuses a library built from other sources or settings."""
    from warehouse import _native

    return _native.tree_source_sha()


def load_profile(tag):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))[tag]
    except Exception:
        return None
    return d if d.get("source_sha") == source_sha() else None


def load_traffic(tag, launches_bytes=None):
    d = load_profile(tag)
    return None if d is None else d.get("bytes_per_launch")


def config_name(variant, na, envs, policy):
    """BASELINE.json config this run corresponds to (SURVEY §8 notation), else 'custom'."""
    known = {("small", 4, 4096, "random"): "C2", ("medium", 8, 65536, "greedy"): "C3",
             ("large", 16, 65536, "greedy"): "C4"}
    return known.get((variant, na, envs, policy), "custom")


def load_issue(tag, steps_per_launch):
    """VALU issue view of the step kernel from the committed SQ counters (profiles/pmc_traffic.json,
    same kernel sources only): per wave and env-step, VALU instructions and wave quad-cycles.
    `single_wave_issue_occupancy` = VALU per wave quad-cycle: the share of the issue slots ONE wave
    can use (one VALU per 4 cycles) that it fills -- an occupancy, not a roofline fraction (two waves
    per SIMD could issue twice as many; the chip-level fraction is roofline.valu)."""
    d = load_profile(tag)
    try:
        sq = d["sq"]
        spl = d.get("steps_per_launch", steps_per_launch)
        waves = sq["SQ_WAVES"]
        valu = sq["SQ_INSTS_VALU"] / waves / spl
        cyc = sq["SQ_WAVE_CYCLES"] / waves / spl
        return {"valu_per_wave_step": valu, "wave_quad_cycles_per_step": cyc,
                "single_wave_issue_occupancy": valu / cyc,
                "wait_quad_cycles_per_step": sq.get("SQ_WAIT_ANY", 0.0) / waves / spl,
                "lds_per_wave_step": sq["SQ_INSTS_LDS"] / waves / spl,
                "source": f"profiles/pmc_traffic.json:{tag}.sq ({spl} steps per launch)"}
    except Exception:
        return None


def valu_roofline(prof, kernel_ms):
    """The chip-level VALU roofline of a kernel: SQ_INSTS_VALU per launch (same-sha SQ profile) / the
    launch's duration / VALU_PEAK_GIPS.  `frac` uses the live HIP-event duration of the timed launch,
    `frac_rocprof` the profile's own kernel-trace average.  None without a same-sha SQ profile."""
    try:
        v = prof["sq"]["SQ_INSTS_VALU"]
    except (TypeError, KeyError):
        return None
    out = {"valu_per_launch": v, "achieved": v / (kernel_ms * 1e-3) / 1e9, "peak": VALU_PEAK_GIPS,
           "unit": "G wave64-VALU/s", "frac": v / (kernel_ms * 1e-3) / 1e9 / VALU_PEAK_GIPS,
           "peak_basis": f"{SIMDS} SIMDs x 2.4 GHz / 2 cycles per wave64 VALU (MI355X_MICROARCH.md)"}
    if prof.get("avg_ns"):
        out["rocprof_avg_ms"] = prof["avg_ns"] * 1e-6
        out["frac_rocprof"] = v / (prof["avg_ns"] * 1e-9) / 1e9 / VALU_PEAK_GIPS
    return out


# ----------------------------------------------------------------------------- multi-GPU plumbing
def rank_info(environ=None):
    """(world, rank, local_rank) from the torch.distributed.run environment (1, 0, 0 without it)."""
    env = os.environ if environ is None else environ
    return int(env.get("WORLD_SIZE", "1")), int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def check_world(gpus, environ=None):
    """--gpus N against the launcher's environment.  Returns "launch" when this process must start the
    N ranks itself (no WORLD_SIZE and N > 1), "run" otherwise; a WORLD_SIZE that differs from --gpus
    is an error (the line would report a world size the command did not ask for)."""
    env = os.environ if environ is None else environ
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher's WORLD_SIZE is {ws}; they must agree")
    return "run"


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(gpus, argv, environ=None, port=None):
    """`python bench.py --gpus N` without a launcher: start N child processes of this script, one per
    GPU, with torch.distributed.run's variables (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
    MASTER_PORT), wait for all of them and return the worst exit code.  The parent has imported
    neither torch nor the library when it gets here: nothing in this process touches a GPU, and the
    children are started as new processes (no exec).  Rank 0 prints the single JSON line.  If one
    rank fails, the others (blocked in a barrier) are terminated by PID."""
    import subprocess

    base = dict(os.environ if environ is None else environ)
    port = port or _free_port()
    procs = []
    for r in range(gpus):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WH_BENCH_SELF_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [None] * gpus
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def assign_device(local, world, device_count, shared_ok):
    """The GPU of a rank: LOCAL_RANK, one per card.  A node with fewer cards than ranks is an error
    unless the run is an explicit rehearsal (--rehearse-shared-devices), where ranks share cards
    round-robin and the line says so (physical_devices, devices_shared).  Returns (index, shared)."""
    if device_count < 1:
        raise SystemExit("bench.py: no GPU visible")
    if local < device_count:
        return local, world > device_count
    if not shared_ok:
        raise SystemExit(f"bench.py: rank {local} needs a GPU of its own but the node has {device_count}; "
                         "pass --rehearse-shared-devices for a rehearsal on shared cards (not a scaling measurement)")
    return local % device_count, True


# Environment switches the library reads that change which kernels run (A/B experiments).  A bench
# line measured with one set does not describe the production path: refused unless --allow-overrides,
# and recorded in the line either way.
KERNEL_OVERRIDES = ("WH_SAMPLER_UNFUSED", "WH_MLP_LEGACY", "WH_MLP_ABLATE", "WH_ABLATE", "WAREHOUSE_AMD_LIB",
                    "WAREHOUSE_AMD_AB")


def kernel_overrides(environ=None):
    env = os.environ if environ is None else environ
    return {k: env[k] for k in KERNEL_OVERRIDES if k in env}


def shard_offset(rank, envs_per_gpu):
    """Rank r owns global env ids [r*B, (r+1)*B): philox draws are keyed by global id, so the shards
    together run exactly the trajectories of one batch of world*B envs (no collective needed)."""
    return rank * envs_per_gpu


# Lead time of the common start: rank 0 names a start instant this far ahead on the node's monotonic
# clock and every rank spins until it, so the ranks' windows open within microseconds of each other
# (a barrier alone releases them tens of microseconds apart -- as long as a short timed window).
START_LEAD_S = 0.005


class WindowTime(float):
    """Seconds of the union window [earliest start, latest end] over the ranks -- what every rank's
    shard was processed in, so `units of all ranks / this` is the whole job's rate -- carrying each
    rank's own window on the node's shared monotonic clock (time.perf_counter is CLOCK_MONOTONIC:
    one clock for every process on the node)."""

    def __new__(cls, starts, ends):
        w = float.__new__(cls, max(ends) - min(starts))
        w.starts, w.ends = list(starts), list(ends)
        return w

    @property
    def per_rank(self):
        return [e - s for s, e in zip(self.starts, self.ends)]

    @property
    def overlap(self):
        """Fraction of the union window in which every rank's window was open."""
        common = min(self.ends) - max(self.starts)
        return max(0.0, common) / float(self) if float(self) > 0 else 1.0

    def describe(self, units_per_rank=None):
        t0 = min(self.starts)
        out = {"union_s": float(self), "max_rank_s": max(self.per_rank), "per_rank_s": self.per_rank,
               "rank_start_offsets_us": [(s - t0) * 1e6 for s in self.starts],
               "rank_end_offsets_us": [(e - t0) * 1e6 for e in self.ends],
               "overlap_frac": self.overlap,
               "note": "value = units of all ranks / union_s (the union of the ranks' windows on the node's "
                       "monotonic clock); per_rank_s are the ranks' own windows, overlap_frac the share of "
                       "the union in which all of them were open"}
        if units_per_rank is not None:
            out["per_rank_rate"] = [units_per_rank / w for w in self.per_rank]
        return out


def timed_window(run, sync, world, dist, start_delay=0.0):
    """The contract's timing window: barrier + device sync on both sides of `run`, all ranks starting
    at a common instant (rank 0 broadcasts it; START_LEAD_S ahead), each rank's [start, end] taken on
    the node's shared monotonic clock and gathered (gloo; nothing on the data path).  Returns a
    WindowTime: the union window, >= the slowest rank's own window (the contract's max over ranks).
    start_delay: seconds this rank waits past the common start (tests: deliberately skewed ranks)."""
    if world > 1:
        import torch

        dist.barrier()
    sync()
    if world > 1:
        at = torch.tensor([time.perf_counter() + START_LEAD_S], dtype=torch.float64)
        dist.broadcast(at, src=0)
        start_at = float(at.item())
        while time.perf_counter() < start_at:
            pass
    if start_delay:
        time.sleep(start_delay)
    t0 = time.perf_counter()
    run()
    sync()
    t1 = time.perf_counter()
    if world == 1:
        return WindowTime([t0], [t1])
    dist.barrier()
    mine = torch.tensor([t0, t1], dtype=torch.float64)
    allw = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allw, mine)
    return WindowTime([float(w[0]) for w in allw], [float(w[1]) for w in allw])


def aggregate_rate(world, envs_per_gpu, agents, steps, elapsed):
    """Whole-job agent-steps/s: every rank stepped its B envs x agents for `steps` steps inside the
    union of the ranks' windows (timed_window)."""
    return world * envs_per_gpu * agents * steps / elapsed


def window_setup_steps(T, K, pre):
    """Untimed positioning steps so that the timed window, which starts after `pre` other steps
    (capture warm-up, the dry run, the warmup), is centred on an episode end (t = T: done,
    auto-reset, and the expiry of the reset-time requests, core.py:303-306, 438):
    setup + pre + K//2 = T (mod T)."""
    return (T - (K // 2) % T - pre) % T


def launch_plan(K, chunk):
    """Steps per fused launch covering K steps."""
    plan = [chunk] * (K // chunk)
    if K % chunk:
        plan.append(K % chunk)
    return plan


def measure(env, mode, policy, K, W, chunk, dev, world, dist, position=True):
    """Time K steps of `mode` (the contract's window).  The kernel time comes from HIP events recorded
    on the launch stream INSIDE that window around exactly the timed launches, so the roofline
    describes the launches that were timed.  Before the warmup, one untimed dry run of the same
    launches, events and synchronisation warms the host path (it is part of the setup steps).
    Returns a dict."""
    import torch

    B, NA = env.B, env.agent_slots
    T = int(env.geometry["T"])
    stream = torch.cuda.current_stream(dev)
    whole = K * B * (NA * 4 + 1) <= (4 << 30)     # per-step outputs of the whole window fit: keep them all
    pre = 0
    if mode == "graph":
        rew1 = torch.zeros((1, B, NA), device=dev)
        dn1 = torch.zeros((1, B), dtype=torch.uint8, device=dev)

        def one():   # reads the current stream per call: the capture runs on a side stream
            env.rollout(1, policy, 0.0, rewards=rew1, dones=dn1)

        for _ in range(3):
            one()
        pre += 3
        torch.cuda.synchronize(dev)
        G = min(K, 200)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                one()
        # capture replays nothing: the G captured steps run only when replayed
        torch.cuda.synchronize(dev)
        tail = env.rollout_launcher(1, policy, 0.0, rewards=rew1, dones=dn1)
        launches = [graph.replay] * (K // G) + [tail] * (K % G)
        plan = [1] * K
        dn = None
    else:
        plan = launch_plan(K, chunk)
        if whole:
            rew = torch.zeros((K, B, NA), device=dev)
            dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
        else:
            rew = torch.zeros((chunk, B, NA), device=dev)
            dn = torch.zeros((chunk, B), dtype=torch.uint8, device=dev)
        launches, off = [], 0
        for c in plan:
            o = off if whole else 0
            launches.append(env.rollout_launcher(c, policy, 0.0, rewards=rew[o:o + c], dones=dn[o:o + c]))
            off += c
    # (events attached to the dispatch itself, wh_launch_run_timed, measured 7 us MORE window time per
    # launch than these two marker records: tools/launch_cost.py)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        ev0.record(stream)
        for launch in launches:
            launch()
        ev1.record(stream)

    timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)     # dry run (setup)
    pre += K
    setup = window_setup_steps(T, K, pre + W) if position else 0
    if setup:
        env.rollout(setup, policy, 0.0)           # position the window (untimed, no outputs)
    if W:
        wr = torch.zeros((min(W, chunk), B, NA), device=dev)
        wd = torch.zeros((min(W, chunk), B), dtype=torch.uint8, device=dev)
        for c in launch_plan(W, chunk):
            env.rollout(c, policy, 0.0, rewards=wr[:c], dones=wd[:c])
        del wr, wd
    elapsed = timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)
    span_ms = ev0.elapsed_time(ev1)
    kernels = len(plan)
    bytes_total = sum(B * (2 * 4 * env.layout.words_per_env + c * (4 * NA + 1)) for c in plan)
    dones = int(dn.sum().item()) if (dn is not None and whole) else None
    start = (pre + setup + W) % T
    return dict(elapsed=elapsed, window=elapsed.describe(B * NA * K), span_ms=span_ms, kernel_ms=span_ms / kernels,
                launches=kernels,
                steps_per_launch=plan[0], bytes_per_launch=bytes_total / kernels,
                achieved_gbs=bytes_total / (span_ms * 1e-3) / 1e9, bytes_per_env_step=bytes_total / (B * K),
                host_fixed_us=(elapsed * 1e3 - span_ms) * 1e3, setup_steps=pre + setup,
                window_t=[start, (start + K) % T], dones_in_window=dones)


def measure_sampler(env, K, W, dev, world, dist):
    """The RLlib sampler route (scripts/train.py's workload): per step the device greedy policy
    stands in for the learner's policy -- BatchedWarehouse.sampler_step = wh_sampler_step: policy +
    step + auto-reset + observation rows [B,NA,9R+1] f32 in ONE launch (k_sampler).  hipGraph of G
    steps.  Returns (elapsed_s, {kernel: ms per launch}) with each launch form timed alone between
    HIP events on the launch stream (20 back-to-back launches): the fused launch, and for comparison
    the two-launch form it replaces (the 1-step fused-rollout launch, then wh_observe)."""
    import torch

    stream = torch.cuda.current_stream(dev)

    def one():
        env.sampler_step("greedy", 0.0, observe=True)

    for _ in range(max(W, 3)):
        one()
    torch.cuda.synchronize(dev)
    G = min(K, 100)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            one()
    torch.cuda.synchronize(dev)

    def run():
        for _ in range(K // G):
            graph.replay()
        for _ in range(K % G):
            one()

    elapsed = timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)

    def per_launch(fn):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in evs:
            a.record(stream)
            for _ in range(20):
                fn()
            b.record(stream)
        torch.cuda.synchronize(dev)
        kms = sorted(a.elapsed_time(b) / 20 for a, b in evs)
        return kms[len(kms) // 2]

    # the write ceiling of the rows: a plain fill_ of a buffer of the same size (the same bytes,
    # streamed with nothing to compute), timed the same way
    rows = torch.empty((env.B, env.agent_slots, env.obs_len), device=dev)
    split = {"sampler_step": per_launch(one),
             "step_only": per_launch(lambda: env.sampler_step("greedy", 0.0, observe=False)),
             "observe_only": per_launch(env.observe),
             "write_ceiling": per_launch(lambda: rows.fill_(1.0))}
    # The env-owned rows are rewritten in place every step (the sampler API's buffer), so at Medium-8
    # (172 MB) they stay in the 256 MB last-level cache (MALL).  The same launches writing a ring of
    # ROT buffers (> 600 MB: fresh HBM every step), and the fill_ of that ring, are the HBM figures.
    ROT = 4
    ring = [torch.empty_like(rows) for _ in range(ROT)]
    own = env._obs
    state = {"i": 0}

    def one_rot():
        env._obs = ring[state["i"] % ROT]
        state["i"] += 1
        env.sampler_step("greedy", 0.0, observe=True)

    def fill_rot():
        ring[state["i"] % ROT].fill_(1.0)
        state["i"] += 1

    split["sampler_step_rotating"] = per_launch(one_rot)
    split["write_ceiling_rotating"] = per_launch(fill_rot)
    env._obs = own
    del rows, ring
    split["rotating_buffers"] = ROT
    return elapsed, split


def sampler_fused(env):
    """Whether wh_sampler_step runs as one k_sampler launch for env's shape (warehouse_amd.hip
    wh_sampler_step: the fast step instance -- every slot live, even agent count -- and at most 4 KB of
    rows per env, fuse_rows; Large builds no k_sampler, kSamplerBuilt), else the step launch + k_observe."""
    NA = env.agent_slots
    return (NA % 2 == 0 and env.layout.kernel_agents == NA and not env.train
            and 4 * NA * env.obs_len <= 4096 and int(env.geometry["R"]) < 16)


def sampler_line(env, Ks, el, split, world, variant, words, fused):
    """The bench line of the sampler route at env's shape (measure_sampler's numbers): throughput,
    the per-launch split and the roofline of the launch that writes the rows.  fused: one k_sampler
    launch per step (Medium-8); else the step launch + k_observe (configurations whose fused step
    would spill at two waves per SIMD, Large-16)."""
    B, NA = env.B, env.agent_slots
    fms = split["sampler_step"]
    rows_b = B * NA * env.obs_len * 4
    # algorithmic bytes of a sampler step: rows written + packed state read and written (twice for
    # the two-launch form: the observation launch reads it again) + rewards + dones
    samp_b = rows_b + (2 if fused else 3) * B * 4 * words + B * (4 * NA + 1)
    kname = "k_sampler" if fused else "k_step (1 step) + k_observe"
    out = {
        "workload": f"RLlib sampler route, {variant} N={NA}, B={B}: device greedy policy + step + auto-reset + f32 "
                    f"observation rows [B,{NA},{env.obs_len}] per step (wh_sampler_step -> "
                    f"{'one k_sampler launch' if fused else 'k_step + k_observe'}); hipGraph of 100 steps",
        "value": aggregate_rate(world, B, NA, Ks, el), "unit": "agent-steps/s", "steps": Ks,
        "ms_per_step": el * 1e3 / Ks,
        "kernel_split_ms": {
            (f"{kname} (greedy + step + auto-reset + rows)"): fms,
            "two-launch form: k_step (1-step rollout)": split["step_only"],
            "two-launch form: k_observe": split["observe_only"],
            f"write ceiling: torch fill_ of the same {rows_b / 1e6:.1f} MB": split["write_ceiling"]},
        "two_launch_form_ms": split["step_only"] + split["observe_only"],
        # what the step costs on top of streaming the same rows: the sampler launch minus a plain
        # write of the same bytes (and, for comparison, minus k_observe, which also builds the rows)
        "step_share_ms": fms - split["write_ceiling"],
        "step_share_vs_observe_ms": fms - split["observe_only"],
        "roofline": {"bound": "hbm", "kernel": kname, "kernel_ms": fms,
                     "bytes_per_launch": samp_b, "achieved": samp_b / (fms * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": samp_b / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "write_ceiling_frac": rows_b / (split["write_ceiling"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "footprint": (f"{rows_b / 1e6:.0f} MB of rows rewritten in place every step (the env-owned "
                                   f"buffer): " + ("it fits the 256 MB last-level cache (MALL), so `frac` is a "
                                                   "cache-resident rate, not HBM" if rows_b < 256e6 else
                                                   "larger than the 256 MB last-level cache: HBM")),
                     "note": "algorithmic bytes = B*NA*(9R+1)*4 rows + packed state (read + write, + a second "
                             "read for the two-launch form) + rewards + dones; write_ceiling_frac = the rows' bytes "
                             "/ the fill_ time / 8 TB/s"},
    }
    if "sampler_step_rotating" in split:
        rms, rot = split["sampler_step_rotating"], split["rotating_buffers"]
        out["roofline_rotating"] = {
            "bound": "hbm", "kernel": kname, "kernel_ms": rms, "bytes_per_launch": samp_b,
            "achieved": samp_b / (rms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": samp_b / (rms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "write_ceiling_ms": split["write_ceiling_rotating"],
            "write_ceiling_frac": rows_b / (split["write_ceiling_rotating"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "vs_write_ceiling": split["write_ceiling_rotating"] / rms,
            "footprint": f"the same launches writing a ring of {rot} row buffers ({rot * rows_b / 1e6:.0f} MB): every "
                         "step's rows go to memory the last-level cache does not hold -- the HBM figure"}
    return out


def measure_sampler_rollout(env, K, frag, W, dev, world, dist):
    """The sampler route as rollout fragments (wh_sampler_rollout): `frag` sampler steps per launch,
    the obs rows / rewards / dones of every step kept ([frag,B,NA,9R+1] ...), K steps in the timed
    window.  Returns (elapsed_s, ms per launch timed alone between HIP events)."""
    import torch

    stream = torch.cuda.current_stream(dev)
    B, NA = env.B, env.agent_slots
    obs = torch.empty((frag, B, NA, env.obs_len), device=dev)
    rew = torch.empty((frag, B, NA), device=dev)
    dn = torch.empty((frag, B), dtype=torch.uint8, device=dev)

    def one():
        env.sampler_rollout(frag, "greedy", 0.0, obs=obs, rewards=rew, dones=dn)

    for _ in range(max(W // frag, 2)):
        one()
    torch.cuda.synchronize(dev)
    n = max(1, K // frag)

    def run():
        for _ in range(n):
            one()

    elapsed = timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        one()
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) for a, b in evs)
    del obs
    return elapsed, n * frag, kms[len(kms) // 2]


def measure_vector(env, K, W, dev, world, dist, order=None):
    """The RLlib route with the learner's actions (scripts/train.py's MultiAgentEnv sampler, through
    WarehouseVectorEnv): per step wh_vector_step = external actions [B,NA] -> step + auto-reset +
    observation rows, one launch (k_sampler's generic instance).  The actions are one fixed tensor
    (the learner's forward pass is not part of the env step).  hipGraph of G steps.  Returns
    (elapsed_s, ms per launch timed alone between HIP events)."""
    import torch

    stream = torch.cuda.current_stream(dev)
    acts = env.policy("greedy", 0.0).clone()

    def one():
        env.vector_step(acts, autoreset=True, order=order)

    for _ in range(max(W, 3)):
        one()
    torch.cuda.synchronize(dev)
    G = min(K, 100)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(G):
            one()
    torch.cuda.synchronize(dev)

    def run():
        for _ in range(K // G):
            graph.replay()
        for _ in range(K % G):
            one()

    elapsed = timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        for _ in range(20):
            one()
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) / 20 for a, b in evs)
    return elapsed, kms[len(kms) // 2]


def measure_sampler_pipeline(env, K, W, dev, world, dist):
    """The same sampler route as a two-stream pipeline (warehouse.vector.SamplerPipeline): step s + 1
    (wh_sampler_step_to, double-buffered state) on the launch stream while the observation rows of
    step s are written on a side stream -- the same launches and results as measure_sampler's.
    hipGraph of G (even) steps.  Returns elapsed_s."""
    import torch

    from warehouse.vector import SamplerPipeline

    pipe = SamplerPipeline(env, "greedy", 0.0)
    pipe.begin()
    for _ in range(max(W, 4)):
        pipe.step()
    pipe.end()
    torch.cuda.synchronize(dev)
    G = 100 if K >= 100 else max(2, K - K % 2)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        pipe.begin()
        for _ in range(G):
            pipe.step()
        pipe.end()
    torch.cuda.synchronize(dev)
    reps = max(1, K // G)

    def run():
        for _ in range(reps):
            graph.replay()

    return timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist), reps * G


def measure_policy(env, K, W, dev, world, dist, precision="bf16"):
    """scripts/rollout.py's loop on the device: per step the SAC policy network
    (wh_mlp_forward, argmax) over all B x NA observation rows, then the step (step +
    auto-reset + next rows: wh_vector_step_x for the bf16 network's fragment operand,
    wh_vector_step's f32 rows for the f32 network).  hipGraph of G steps.  Returns (elapsed_s, mlp_kernel_ms, net)."""
    import torch

    import warehouse.policy as wp

    net = wp.MLPPolicy(env.variant, seed=7, device=dev, precision=precision)
    B, NA = env.B, env.agent_slots
    acts = torch.empty((B, NA), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    # bf16: the observation rows go to the network as its layer-0 operand (wh_observe_x, bf16 in
    # MFMA fragment order; the same inputs as rounding the f32 rows) -- nothing else reads them on
    # this route; f32: the float32 rows
    frag = precision == "bf16"
    obs = env.observe_x() if frag else env.observe()

    def infer():
        if frag:
            net.forward_x(obs, B * NA, step=0, actions=acts.view(-1))
        else:
            net(obs.view(B * NA, -1), step=0, actions=acts.view(-1))

    def one():
        infer()
        if frag:   # step + the next operand (wh_vector_step_x)
            env.vector_step_x(acts, autoreset=True)
        else:
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

    def run():
        for _ in range(K // G):
            graph.replay()
        for _ in range(K % G):
            one()

    elapsed = timed_window(run, lambda: torch.cuda.synchronize(dev), world, dist)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in evs:
        a.record(stream)
        for _ in range(5):
            infer()
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = sorted(a.elapsed_time(b) / 5 for a, b in evs)
    return elapsed, kms[len(kms) // 2], net


def mlp_kernel_name(net, prec):
    """The policy kernel wh_mlp_forward dispatches for this network (policy_mlp.hip find_mlp): the
    exact-f32 kernel, or bf16 on 16x16x32 tiles (k_mlp16) for the Medium and Large shapes, else the
    32x32x16 kernel (k_mlp)."""
    if prec != "bf16":
        return "k_mlp_f32"
    if (net.in_dim, net.hidden[0], net.hidden[1]) in ((82, 512, 512), (145, 1024, 256)):
        return "k_mlp16 (v_mfma_f32_16x16x32_bf16)"
    return "k_mlp (v_mfma_f32_32x32x16_bf16)"


def profile_tag(variant, NA, policy, envs, mode, steps_per_launch):
    """The profiles/pmc_traffic.json key of a step-kernel launch shape: the C3/C4 greedy shapes at
    B = 65,536 keep their short keys, other shapes name policy and batch."""
    if policy == "greedy" and envs == 65536:
        return f"{variant}_n{NA}_{mode}_k{steps_per_launch}"
    return f"{variant}_n{NA}_{policy}_b{envs}_{mode}_k{steps_per_launch}"


def config_leg(name, variant, NA, B, policy, K, W, chunk, dev, world, dist, rank):
    """Another BASELINE config through the headline's own measurement (measure(): one prepared launch
    of K fused steps -- policy + step + auto-reset, rewards and dones written -- timed inside the
    contract's window, placed across an episode end), with its own roofline."""
    import warehouse

    env = warehouse.BatchedWarehouse(variant, B, NA, seed=1234, env_offset=shard_offset(rank, B), device=dev)
    env.reset()
    m = measure(env, "fused", policy, K, W, chunk, dev, world, dist)
    return {"workload": f"{name}: {variant} N={NA}, B={B} envs/GPU, {policy} policy fused with step + auto-reset, "
                        f"{m['launches']} launch(es) of {m['steps_per_launch']} steps",
            "value": aggregate_rate(world, B, NA, K, m["elapsed"]), "unit": "agent-steps/s", "steps": K,
            "ms_per_step": m["elapsed"] * 1e3 / K, "window": m["window"],
            "dones_in_window": m["dones_in_window"],
            "roofline": step_roofline(m, variant, NA, policy, "fused", B)}


def vector_leg(env, K, W, dev, world, dist, label, order=None):
    """wh_vector_step (external actions, auto-reset, f32 rows) at env's shape: throughput and the
    HBM roofline of the launch(es) per step."""
    B, NA = env.B, env.agent_slots
    el, vms = measure_vector(env, K, W, dev, world, dist, order=order)
    words = env.layout.words_per_env
    fused = sampler_fused(env) or (order is not None and 4 * NA * env.obs_len <= 4096 and NA % 2 == 0
                                   and int(env.geometry["R"]) < 16)
    vec_b = (B * NA * env.obs_len * 4 + (2 if fused else 3) * B * 4 * words + B * (4 * NA + 1) + B * NA * 4
             + (0 if order is None else 4 * order.numel()))
    return {"workload": label, "value": aggregate_rate(world, B, NA, K, el), "unit": "agent-steps/s", "steps": K,
            "ms_per_step": el * 1e3 / K,
            "roofline": {"bound": "hbm", "kernel": "k_sampler<external actions>" if fused else "k_step + k_observe",
                         "kernel_ms": vms, "bytes_per_launch": vec_b, "achieved": vec_b / (vms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": vec_b / (vms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "algorithmic bytes = rows + packed state (read + write, + a second read for two "
                                 "launches) + rewards + dones + actions (+ order rows)"}}


def step_roofline(m, variant, NA, policy, mode, envs):
    """The bench line's `roofline` for the timed launches of measure() (dict m).  achieved / peak /
    frac are the contract's HBM figures (algorithmic bytes per launch / the launch's event-timed
    duration, against 8 TB/s); `valu` is the chip-level VALU issue roofline of the same launch (from
    the same-sha SQ profile), and `bound` names whichever of the two fractions is higher -- the
    step kernel keeps its state in registers and is VALU-issue bound."""
    tag = profile_tag(variant, NA, policy, envs, mode, m["steps_per_launch"])
    prof = load_profile(tag)
    hbm_frac = m["achieved_gbs"] / HBM_PEAK_GBS
    valu = valu_roofline(prof, m["kernel_ms"])
    bound = "valu" if valu is not None and valu["frac"] > hbm_frac else "hbm"
    return {
        "bound": bound,
        "achieved": m["achieved_gbs"],
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": hbm_frac,
        "hbm_frac": hbm_frac,
        "valu_frac": None if valu is None else valu["frac"],
        "valu": valu,
        "traffic": None if prof is None else prof.get("bytes_per_launch"),
        "kernel": f"k_step<Cfg<D,R,racks,{NA}>, {policy}>",
        "kernel_ms": m["kernel_ms"],
        "launches": m["launches"],
        "steps_per_launch": m["steps_per_launch"],
        "bytes_per_launch": m["bytes_per_launch"],
        "bytes_per_env_step": m["bytes_per_env_step"],
        "host_fixed_us": m["host_fixed_us"],
        "rocprof_avg_ms": None if prof is None or prof.get("avg_ns") is None else prof["avg_ns"] * 1e-6,
        "issue": load_issue(tag, m["steps_per_launch"]),
        "profile": None if prof is None else f"profiles/pmc_traffic.json:{tag}",
        "note": "achieved/peak/frac: HBM (algorithmic bytes = 2 x packed state + per-step rewards/dones, per "
                "launch / kernel_ms); valu: SQ_INSTS_VALU of the same launch shape / kernel_ms against "
                "1,024 SIMDs x 1.2 G wave64-VALU/s; bound = the larger fraction.  kernel_ms = HIP-event "
                "span of the timed launches / launches (events on the launch stream inside the timed "
                "window); host_fixed_us = window wall time - that span (launch + completion latency)",
    }


def report(out, args):
    """Rank 0's line: `out` plus the host-core baseline of the same workload (cpu_baseline: the numpy
    restatement of Warehouse.step() on a bounded sample, one process per host core), timed after the
    GPU window at EVERY world size, so a 1/2/4/8-GPU run carries the host-core figure of the same run.
    Prints the JSON line and returns it."""
    if not args.no_cpu_baseline:
        cores, detail = host_cores()
        procs = args.cpu_procs or cores
        out["cpu_baseline"] = cpu_baseline(args.variant, args.agents, procs, args.cpu_seconds, detail)
        out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)
    return out


def plumbing_only(args, world, rank, dist):
    """--plumbing-only: the multi-rank path end to end without a GPU (CPU tests of the self-launch):
    gloo group, shard offsets, the barrier/max timing window around a host-side sleep, the aggregate
    and rank 0's line with the host-core baseline.  No kernel runs; the line says so."""
    if world > 1:
        dist.init_process_group("gloo")
    B, NA, K = args.envs, args.agents, args.steps
    elapsed = timed_window(lambda: time.sleep(0.05 * (rank + 1)), lambda: None, world, dist)
    if world > 1:
        import torch

        offs = torch.tensor([shard_offset(rank, B)], dtype=torch.int64)
        gathered = [torch.zeros_like(offs) for _ in range(world)]
        dist.all_gather(gathered, offs)
        offsets = [int(g.item()) for g in gathered]
    else:
        offsets = [0]
    if rank == 0:
        report({"metric": f"PLUMBING SELF-TEST, NOT A MEASUREMENT ({METRIC})",
                "value": aggregate_rate(world, B, NA, K, elapsed), "unit": "agent-steps/s", "n_gpus": world,
                "steps": K, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / K, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "none", "data": "none: no kernel ran",
                "window": elapsed.describe(B * NA * K),
                "config": {"workload": "plumbing self-test", "envs_per_gpu": B, "agents": NA,
                           "shard_offsets": offsets,
                           "launch": "self-launched ranks" if os.environ.get("WH_BENCH_SELF_LAUNCHED") else
                                     ("launcher" if world > 1 else "single process")}}, args)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


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
    ap.add_argument("--no-desync", action="store_true", help="skip the desynchronised-episodes measurement")
    ap.add_argument("--no-policy", action="store_true", help="skip the SAC-policy rollout measurement")
    ap.add_argument("--no-configs", action="store_true", help="skip the C2 / C4 legs")
    ap.add_argument("--policy-steps", type=int, default=200)
    ap.add_argument("--policy-steps-f32", type=int, default=40)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = one per host core (host_cores())")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse-shared-devices", action="store_true",
                    help="allow more ranks than GPUs (ranks share cards round-robin): a rehearsal of the "
                         "N > 1 path, flagged in the line, not a scaling measurement")
    ap.add_argument("--allow-overrides", action="store_true",
                    help="run even when an A/B kernel-selection variable (KERNEL_OVERRIDES) is set")
    ap.add_argument("--plumbing-only", action="store_true",
                    help="self-test of the multi-rank plumbing without a GPU: no kernel runs, the window "
                         "times a host-side sleep; the line is marked as such")
    args = ap.parse_args()

    # N ranks without a launcher: start them from here, before anything touches a GPU
    if check_world(args.gpus) == "launch":
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    overrides = kernel_overrides()
    if overrides and not args.allow_overrides and not args.plumbing_only:
        raise SystemExit(f"bench.py: kernel-selection overrides set {overrides}; unset them or pass --allow-overrides")

    import torch
    import torch.distributed as dist

    world, rank, local = rank_info()
    if args.plumbing_only:
        return plumbing_only(args, world, rank, dist)
    # one GPU per rank (device_count() initialises nothing on this image)
    ndev = torch.cuda.device_count()
    local, shared = assign_device(local, world, ndev, args.rehearse_shared_devices)
    torch.cuda.set_device(local)             # before any other GPU call of this rank
    if world > 1:
        dist.init_process_group("gloo")
    dev = torch.device("cuda", local)

    import warehouse
    from warehouse import _native

    # provenance: the loaded library must have been built from this tree's kernel sources
    binary_sha = _native.verify_provenance()

    B, NA, K, W = args.envs, args.agents, args.steps, args.warmup
    env = warehouse.BatchedWarehouse(args.variant, B, NA, seed=1234, env_offset=shard_offset(rank, B), device=dev)
    env.reset()

    m = measure(env, args.mode, args.policy, K, W, args.chunk, dev, world, dist)
    value = aggregate_rate(world, B, NA, K, m["elapsed"])
    alt = None
    if not args.no_alt:
        other = "graph" if args.mode == "fused" else "fused"
        env.reset()
        m2 = measure(env, other, args.policy, K, W, args.chunk, dev, world, dist)
        alt = {"mode": other, "value": aggregate_rate(world, B, NA, K, m2["elapsed"]),
               "ms_per_step": m2["elapsed"] * 1e3 / K, "kernel_ms": m2["kernel_ms"],
               "steps_per_launch": m2["steps_per_launch"], "bytes_per_launch": m2["bytes_per_launch"],
               "roofline_frac": m2["achieved_gbs"] / HBM_PEAK_GBS, "host_fixed_us": m2["host_fixed_us"],
               "traffic": load_traffic(f"{args.variant}_n{NA}_{other}_k{m2['steps_per_launch']}")}

    desync = None
    if not args.no_desync and args.mode == "fused":
        # episodes desynchronised like independent samplers (env e is 37e mod T steps ahead, so the 64
        # lanes of a wave are spread over the episode): every step some lanes of most waves end, reset
        # and run the expiry pass while the others do not
        import numpy as np

        env.reset()
        T = int(env.geometry["T"])
        env.stagger((np.arange(B, dtype=np.int64) * 37) % T)
        # three windows in a row (the episodes stay desynchronised), the median by kernel time: one
        # 20-step window on a box whose clock is settling read anywhere from 1.07x to 1.48x of the
        # synchronised launch with identical code (profiles/r04_desync20_ab.txt)
        runs = [measure(env, "fused", args.policy, K, W, args.chunk, dev, world, dist, position=False) for _ in range(3)]
        md = sorted(runs, key=lambda r: r["kernel_ms"])[1]
        vd = aggregate_rate(world, B, NA, K, md["elapsed"])
        desync = {"workload": "same launches after BatchedWarehouse.stagger: env e is 37e mod T steps ahead, so "
                              "the lanes of every wave are spread over the episode and about B/T envs end "
                              "their episode on every step",
                  "value": vd, "ms_per_step": md["elapsed"] * 1e3 / K, "kernel_ms": md["kernel_ms"],
                  "dones_in_window": md["dones_in_window"], "host_fixed_us": md["host_fixed_us"],
                  "kernel_time_vs_synchronised": md["kernel_ms"] / m["kernel_ms"],
                  "kernel_ms_windows": [r["kernel_ms"] for r in runs]}

    words = env.layout.words_per_env
    sampler = None
    if not args.no_sampler:
        # (at least two replays of the 100-step graph, whatever --steps: the route's steady state,
        # not one graph launch's host latency over a 20-step window)
        Ks = max(min(K, 1000), 200)
        el3, split = measure_sampler(env, Ks, W, dev, world, dist)
        sampler = sampler_line(env, Ks, el3, split, world, args.variant, words, fused=sampler_fused(env))
        sampler["roofline"]["traffic"] = load_traffic(f"{args.variant}_n{NA}_sampler")
        el5, Kpp = measure_sampler_pipeline(env, Ks, W, dev, world, dist)
        sampler["two_stream_pipeline"] = {
            "workload": "the two-launch form as SamplerPipeline: the rows of step s on a side stream while "
                        "step s+1 runs (state double-buffered); slower -- the step launch's workgroups only "
                        "start as the observation kernel's drain (DESIGN.md §5)",
            "value": aggregate_rate(world, B, NA, Kpp, el5), "steps": Kpp, "ms_per_step": el5 * 1e3 / Kpp}

    # C4's shape on the same route (BASELINE config 4: Large, 16 agents, B = 65,536): its step code
    # needs 360 registers, so the fused k_sampler (two waves per SIMD, 256 registers) would spill and
    # the route takes the step launch + k_observe
    sampler_c4 = None
    if not args.no_sampler and (args.variant, NA, B) == ("medium", 8, 65536):
        env4 = warehouse.BatchedWarehouse("large", B, 16, seed=1234, env_offset=shard_offset(rank, B), device=dev)
        env4.reset()
        el8, split8 = measure_sampler(env4, 200, W, dev, world, dist)
        sampler_c4 = sampler_line(env4, 200, el8, split8, world, "large", env4.layout.words_per_env,
                                  fused=sampler_fused(env4))
        del env4

    fragment = None
    if not args.no_sampler:
        frag = 20
        el7, Kf, fms2 = measure_sampler_rollout(env, max(min(K, 1000), 200), frag, W, dev, world, dist)
        frag_b = frag * (B * NA * env.obs_len * 4 + B * (4 * NA + 1)) + 2 * B * 4 * words
        fragment = {
            "workload": f"the sampler route as rollout fragments: wh_sampler_rollout = {frag} sampler steps (device greedy "
                        f"policy + step + auto-reset + f32 observation rows) per launch, every step's rows kept "
                        f"([{frag},B,{NA},{env.obs_len}]); {Kf} steps timed",
            "value": aggregate_rate(world, B, NA, Kf, el7), "unit": "agent-steps/s", "steps": Kf,
            "ms_per_step": el7 * 1e3 / Kf,
            "roofline": {"bound": "hbm", "kernel": f"k_sampler ({frag} steps per launch)", "kernel_ms": fms2,
                         "bytes_per_launch": frag_b, "achieved": frag_b / (fms2 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": frag_b / (fms2 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "algorithmic bytes = per step rows + rewards + dones, + 2 x packed state per launch"},
        }

    vector = None
    if not args.no_sampler:
        Kv = max(min(K, 1000), 200)
        el6, vms = measure_vector(env, Kv, W, dev, world, dist)
        vec_b = B * NA * env.obs_len * 4 + 2 * B * 4 * words + B * (4 * NA + 1) + B * NA * 4
        vector = {
            "workload": f"RLlib route with external actions: wh_vector_step(actions [B,{NA}] int32) = step + "
                        f"auto-reset + f32 observation rows in one launch (k_sampler, generic instance); "
                        f"hipGraph of 100 steps",
            "value": aggregate_rate(world, B, NA, Kv, el6), "unit": "agent-steps/s", "steps": Kv,
            "ms_per_step": el6 * 1e3 / Kv,
            "roofline": {"bound": "hbm", "kernel": "k_sampler<external actions>", "kernel_ms": vms,
                         "bytes_per_launch": vec_b, "achieved": vec_b / (vms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": vec_b / (vms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "algorithmic bytes = rows + 2 x packed state + rewards + dones + actions"},
        }

    # BASELINE configs 2 and 4 through the headline's measurement, in the same run (C3 is the headline)
    legs = {}
    if not args.no_configs and (args.variant, NA, B, args.policy) == ("medium", 8, 65536, "greedy"):
        legs["C2"] = config_leg("C2", "small", 4, 4096, "random", K, W, args.chunk, dev, world, dist, rank)
        legs["C4"] = config_leg("C4", "large", 16, 65536, "greedy", K, W, args.chunk, dev, world, dist, rank)

    # the RLlib route of scripts/train.py's actual env (all three registered names build
    # WarehouseLargeTrain, scripts/train.py:34-35): external actions, n redrawn at every auto-reset
    vector_lt = vector_order = None
    if not args.no_sampler and (args.variant, NA, B) == ("medium", 8, 65536):
        import torch

        envt = warehouse.BatchedWarehouse("large", B, None, train=True, seed=1234, env_offset=shard_offset(rank, B),
                                          device=dev)
        envt.reset()
        vector_lt = vector_leg(envt, 200, W, dev, world, dist,
                               f"scripts/train.py's env (WarehouseLargeTrain: 16 agent slots, n ~ U{{1..16}} per "
                               f"episode), B={B}: wh_vector_step(actions) = step + auto-reset + f32 rows; hipGraph "
                               f"of 100 steps")
        del envt
        # the dict-order kernel (WarehouseBaseEnv with shuffled action dicts): every env's full dict in
        # a fixed random order
        g = torch.Generator(device=dev).manual_seed(7)
        order = torch.argsort(torch.rand((B, NA), device=dev, generator=g), dim=1).to(torch.int32)
        env.reset()
        vector_order = vector_leg(env, 200, W, dev, world, dist,
                                  f"dict-order route (WarehouseBaseEnv.send_actions with shuffled dicts): "
                                  f"wh_vector_step(actions, order) at {args.variant} N={NA}, B={B}, every env's dict "
                                  f"in a random order; hipGraph of 100 steps", order=order)

    policy_line = policy_f32 = None
    if not args.no_policy:
        rows = B * NA
        for prec in ("bf16", "f32"):
            Kp = min(K, args.policy_steps if prec == "bf16" else args.policy_steps_f32)
            el4, mms, net = measure_policy(env, Kp, W, dev, world, dist, prec)
            flop = 2.0 * rows * (net.in_dim * net.hidden[0] + net.hidden[0] * net.hidden[1] + net.hidden[1] * 9)
            peak = MFMA_BF16_PEAK_TFS if prec == "bf16" else MFMA_F32_PEAK_TFS
            line = {
                "workload": f"scripts/rollout.py loop on device: SAC policy_model MLP [{net.in_dim},{net.hidden[0]},"
                            f"{net.hidden[1]},9] argmax over B*NA={rows} rows -> "
                            + ("wh_vector_step_x (step + auto-reset, then the observation rows as the MLP's bf16 "
                               "fragment-order operand)" if prec == "bf16"
                               else "wh_vector_step (step + auto-reset + f32 observation rows)") +
                            "; random-init weights (no checkpoint ships with the reference)",
                "value": aggregate_rate(world, B, NA, Kp, el4), "unit": "agent-steps/s", "steps": Kp,
                "ms_per_step": el4 * 1e3 / Kp,
                "dtype": "bf16 MFMA, f32 accumulate" if prec == "bf16" else "exact f32 MFMA (v_mfma_f32_32x32x2_f32)",
                "roofline": {"bound": "mfma", "kernel": mlp_kernel_name(net, prec), "kernel_ms": mms,
                             "flop_per_launch": flop, "achieved": flop / (mms * 1e-3) / 1e12, "peak": peak,
                             "unit": "TFLOP/s", "frac": flop / (mms * 1e-3) / 1e12 / peak,
                             "traffic": load_traffic(f"{args.variant}_n{NA}_mlp" + ("" if prec == "bf16" else "_f32"))},
            }
            if prec == "bf16":
                policy_line = line
            else:
                policy_f32 = line

    if rank == 0:
        out = {
            "metric": METRIC if not shared else f"{METRIC} [REHEARSAL: {world} ranks shared {ndev} card(s)]",
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": m["elapsed"] * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/u32 packed integer state, f32 rewards",
            "data": "synthetic: philox-seeded episodes keyed by global env id, greedy policy on device",
            "config": {
                "workload": f"{config_name(args.variant, NA, B, args.policy)}: {args.variant} N={NA}, B={B} envs/GPU, "
                            f"{args.policy} policy fused with step + auto-reset (device-resident rollout)",
                "envs_per_gpu": B, "agents": NA, "variant": args.variant, "policy": args.policy,
                "launch": "hipGraph of 1-step launches" if args.mode == "graph" else
                          f"{m['launches']} launch(es) of {m['steps_per_launch']} steps",
                "parallelism": f"independent env shards x{world}, no collectives",
                "window": {"setup_steps": m["setup_steps"], "t_at_start_end": m["window_t"],
                           "dones_in_window": m["dones_in_window"],
                           "note": "untimed setup steps (including one dry run of the timed launches) place "
                                   "the timed window across an episode end (done + auto-reset + request "
                                   "expiry inside it)"},
            },
            "binary": {"wh_version": _native.lib().wh_version().decode(), "source_sha": binary_sha,
                       "tree_source_sha": source_sha(), "path": os.path.relpath(_native.LIB_PATH, ROOT),
                       "kernel_overrides": overrides},
            "devices": {"physical_devices": ndev, "devices_shared": shared,
                        "launch": "self-launched ranks" if os.environ.get("WH_BENCH_SELF_LAUNCHED") else
                                  ("torch.distributed.run" if world > 1 else "single process")},
            "window": m["window"],
            "roofline": step_roofline(m, args.variant, NA, args.policy, args.mode, args.envs),
            "alt_launch_mode": alt,
            "desync_episodes": desync,
            "sampler_path": sampler,
            "sampler_path_c4": sampler_c4,
            "sampler_fragments": fragment,
            "vector_path": vector,
            "vector_path_large_train": vector_lt,
            "vector_path_dict_order": vector_order,
            "config_legs": legs,
            "policy_path": policy_line,
            "policy_path_f32": policy_f32,
        }
        report(out, args)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
