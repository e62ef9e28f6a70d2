"""The multi-GPU path on CPU with gloo, world size 2: bench.py's sharding (rank r owns global env
ids [r*B, (r+1)*B)), its barrier + max-over-ranks timing window, and the shard-invariance contract
(philox draws keyed by global env id) checked with the oracle standing in for each rank's GPU."""
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
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = oc.layout_for("medium")
    ids = np.arange(rank * B, (rank + 1) * B)          # bench.py: env_offset = rank * B
    S = ob.BState.zeros(L, B, 8)
    d = ob.PhiloxDraws(1234, ids)
    ob.reset(L, S, d)
    dist.barrier()
    total = 0.0
    for _ in range(steps):
        rew, done, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        total += float(rew.sum())
        if done.any():
            ob.reset(L, S, d, mask=done)
    elapsed = torch.tensor([float(rank + 1)], dtype=torch.float64)   # stand-in per-rank time
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    pos = torch.from_numpy(S.pos.copy())
    gathered = [torch.zeros_like(pos) for _ in range(world)]
    dist.all_gather(gathered, pos)
    tot = torch.tensor([total], dtype=torch.float64)
    dist.all_reduce(tot)
    if rank == 0:
        np.save(out, np.concatenate([g.numpy() for g in gathered]))
        np.save(out + ".meta.npy", np.array([elapsed.item(), tot.item()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_rank_shards_equal_single_batch(tmp_path):
    B, steps, world = 64, 30, 2
    out = str(tmp_path / "pos.npy")
    mp.start_processes(_worker, args=(world, _free_port(), B, steps, out), nprocs=world, start_method="spawn")
    sharded = np.load(out)
    elapsed, total = np.load(out + ".meta.npy")
    assert elapsed == 2.0                              # max over ranks
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
