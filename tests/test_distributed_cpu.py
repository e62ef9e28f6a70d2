"""The multi-GPU path on CPU with gloo, world size 2, through bench.py's own plumbing: rank_info()
from the torch.distributed.run environment, shard_offset() (rank r owns global env ids
[r*B, (r+1)*B)), timed_window() (barrier + sync on both sides, a common start, the union of the
ranks' windows) and aggregate_rate();
the shard-invariance contract (philox draws keyed by global env id) is checked with the oracle
standing in for each rank's GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import batched as ob
from oracle import core as oc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, B, steps, out):
    import time

    import torch

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    w, r, local = bench.rank_info()
    assert (w, r, local) == (world, rank, rank)
    dist.init_process_group("gloo", rank=r, world_size=w)
    L = oc.layout_for("medium")
    off = bench.shard_offset(r, B)
    ids = np.arange(off, off + B)
    S = ob.BState.zeros(L, B, 8)
    d = ob.PhiloxDraws(1234, ids)
    ob.reset(L, S, d)
    acc = {"total": 0.0}

    def run():
        for _ in range(steps):
            rew, done, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
            acc["total"] += float(rew.sum())
            if done.any():
                ob.reset(L, S, d, mask=done)
        time.sleep(0.2 * (r + 1))        # rank 1 is the slow one: the window is its time

    syncs = []
    elapsed = bench.timed_window(run, lambda: syncs.append(1), w, dist)
    assert len(syncs) == 2                         # device sync on both sides of the window
    rate = bench.aggregate_rate(w, B, 8, steps, elapsed)
    pos = torch.from_numpy(S.pos.copy())
    gathered = [torch.zeros_like(pos) for _ in range(w)]
    dist.all_gather(gathered, pos)
    tot = torch.tensor([acc["total"]], dtype=torch.float64)
    dist.all_reduce(tot)
    if r == 0:
        np.save(out, np.concatenate([g.numpy() for g in gathered]))
        np.save(out + ".meta.npy", np.array([elapsed, tot.item(), rate]))
        # rank 0's line at world size 2 carries the host-core baseline of the same run (bench.report)
        import argparse
        import json

        args = argparse.Namespace(no_cpu_baseline=False, cpu_procs=1, cpu_seconds=0.3, variant="medium", agents=8)
        line = bench.report({"metric": bench.METRIC, "value": rate, "n_gpus": w}, args)
        json.dump(line, open(out + ".line.json", "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_rank_shards_equal_single_batch(tmp_path):
    B, steps, world = 64, 30, 2
    out = str(tmp_path / "pos.npy")
    mp.start_processes(_worker, args=(world, _free_port(), B, steps, out), nprocs=world, start_method="spawn")
    sharded = np.load(out)
    elapsed, total, rate = np.load(out + ".meta.npy")
    assert elapsed >= 0.4                              # max over ranks: rank 1 slept 0.4 s
    assert rate == pytest.approx(world * B * 8 * steps / elapsed)
    import json

    line = json.load(open(out + ".line.json"))
    assert line["n_gpus"] == 2
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] == "port" and "oracle/core.py" in cb["sample"]
    assert line["gpu_over_cpu"] == pytest.approx(rate / cb["value"])
    L = oc.layout_for("medium")
    S = ob.BState.zeros(L, world * B, 8)
    d = ob.PhiloxDraws(1234, np.arange(world * B))
    ob.reset(L, S, d)
    ref_total = 0.0
    for _ in range(steps):
        rew, done, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        ref_total += float(rew.sum())
        if done.any():
            ob.reset(L, S, d, mask=done)
    np.testing.assert_array_equal(sharded, S.pos)
    assert total == ref_total


def _skew_worker(rank, world, port, out):
    """Rank 1 opens its window 0.3 s after the common start and works 0.1 s; rank 0 works 0.2 s from
    the start: the ranks' windows do not overlap at all, the slowest rank's own window is 0.2 s, and
    the union -- what the two shards were processed in -- is ~0.4 s."""
    import json
    import time

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    work = 0.2 if rank == 0 else 0.1
    w = bench.timed_window(lambda: time.sleep(work), lambda: None, world, dist,
                           start_delay=0.0 if rank == 0 else 0.3)
    if rank == 0:
        json.dump({"union": float(w), "rate": bench.aggregate_rate(world, 1000, 8, 10, w),
                   "desc": w.describe(1000 * 8 * 10)}, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_union_window_sets_the_aggregate(tmp_path):
    """bench.timed_window with deliberately skewed ranks: `value` comes from the union of the ranks'
    windows on the shared monotonic clock, not from the slowest rank's own window (which would
    count two serialised windows as concurrent); overlap_frac reports that they never overlapped."""
    import json

    out = str(tmp_path / "w.json")
    mp.start_processes(_skew_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    r = json.load(open(out))
    d = r["desc"]
    assert max(d["per_rank_s"]) == pytest.approx(0.2, abs=0.05)
    assert r["union"] >= 0.39 and r["union"] == pytest.approx(d["union_s"])
    assert r["union"] > max(d["per_rank_s"]) + 0.15
    assert r["rate"] == pytest.approx(2 * 1000 * 8 * 10 / r["union"])
    assert d["overlap_frac"] == 0.0
    assert d["rank_start_offsets_us"][0] == 0.0 and d["rank_start_offsets_us"][1] >= 0.29e6
    assert len(d["per_rank_rate"]) == 2


def test_union_window_of_concurrent_ranks():
    """Two ranks whose windows coincide: union == the slowest rank, overlap 1."""
    import bench

    w = bench.WindowTime([10.0, 10.0], [10.5, 10.4])
    assert float(w) == pytest.approx(0.5) and w.overlap == pytest.approx(0.8)
    w = bench.WindowTime([1.0], [1.25])
    assert float(w) == pytest.approx(0.25) and w.overlap == 1.0


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT") + bench_overrides()}
    env.update(extra)
    return env


def bench_overrides():
    import bench

    return bench.KERNEL_OVERRIDES


@pytest.mark.timeout(600)
def test_bench_self_launches_n_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no torch.distributed.run around it starts both ranks itself (from
    a parent that never touches a GPU), and rank 0 prints ONE line with n_gpus 2, the max-over-ranks
    window and the host-core baseline.  --plumbing-only runs that path with no kernel (CPU here)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing-only",
                        "--steps", "20", "--warmup", "5", "--cpu-procs", "1", "--cpu-seconds", "0.3"],
                       cwd=root, env=_bench_env(), capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and "NOT A MEASUREMENT" in line["metric"]
    assert line["config"]["launch"] == "self-launched ranks"
    assert line["config"]["shard_offsets"] == [0, 65536]
    assert line["ms_per_step"] * 20 >= 100.0          # the window is the slow rank's (0.1 s sleep)
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] == "port"


def test_bench_refuses_a_world_size_other_than_gpus():
    import subprocess
    import sys

    import bench

    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(8, {}) == "launch"
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == "run"
    with pytest.raises(SystemExit):
        bench.check_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.check_world(0, {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing-only"],
                       cwd=root, env=_bench_env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE is 4" in r.stderr


def test_bench_device_assignment_and_overrides():
    import bench

    assert bench.assign_device(3, 8, 8, False) == (3, False)
    assert bench.assign_device(0, 1, 1, False) == (0, False)
    with pytest.raises(SystemExit):
        bench.assign_device(1, 2, 1, False)       # two ranks, one card: not a scaling run
    assert bench.assign_device(1, 2, 1, True) == (0, True)
    assert bench.assign_device(0, 2, 1, True) == (0, True)
    with pytest.raises(SystemExit):
        bench.assign_device(0, 1, 0, False)
    assert bench.kernel_overrides({"WH_SAMPLER_UNFUSED": "1", "PATH": "x"}) == {"WH_SAMPLER_UNFUSED": "1"}
    assert bench.kernel_overrides({}) == {}
