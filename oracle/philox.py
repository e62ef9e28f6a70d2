"""numpy model of the device draw specification ("philox" RNG mode) -- TEST INFRASTRUCTURE ONLY.

The reference draws from numpy's global MT19937 stream, which is inherently sequential and shared
by every env in a process.  The batched device path instead keys a counter-based generator by
(seed, global env id, episode, t), so B envs draw independently and any sharding of env ids over
GPUs reproduces the same trajectories.  This file restates that contract in numpy so the kernels'
philox mode can be checked bit-exactly; the same contract is documented in
include/warehouse_amd.h and DESIGN.md.

    key  = (seed & 0xffffffff, seed >> 32)
    ctr  = (env_id, episode, t, (purpose << 24) | block)
    word(j) of a stream = philox4x32_10(ctr with block = j // 4, key)[j % 4]
    uniform_int(m, w) = (w * m) >> 32

Streams (purpose, t):
  RESET   (1, 0)      word 0: n = 1 + uniform_int(nmax, .) (Train variants only)
                      word 1+i: spawn cell of agent slot i = valid_cells[uniform_int(n_valid, .)]
                      word 1+NA+2j: j-th request pickup by Floyd's algorithm: m = P-R+j,
                                    r = uniform_int(m+1); r unless already chosen, else m
                      word 2+NA+2j: its target = r-th not-yet-chosen delivery point, r = uniform_int(Dp-j)
  REGEN   (2, t_new)  word 2j (j<k): j-th reopened pickup = r-th remaining inactive, r = uniform_int(n_in-j)
                      word 2j+1: its target = r-th target not chosen in this regeneration, r = uniform_int(Dp-j)
  (pickup and target words interleave so the usual k <= 2 reopenings cost one Philox block)
  POLICY  (3, t_obs)  word 2i: coin u = (w >> 8) / 2**24, random iff u < p; word 2i+1: action uniform_int(9)
  RANDOM  (4, t_obs)  word i: action uniform_int(9)
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

RESET, REGEN, POLICY, RANDOM = 1, 2, 3, 4


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11).  Inputs broadcastable uint arrays."""
    c0, c1, c2, c3 = (np.asarray(c, np.uint64) & MASK32 for c in (c0, c1, c2, c3))
    k0 = np.asarray(k0, np.uint64) & MASK32
    k1 = np.asarray(k1, np.uint64) & MASK32
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


class Streams:
    """word(env_ids, episode, t, purpose, j) for arrays of envs."""

    def __init__(self, seed: int):
        self.k0 = np.uint64(seed & 0xFFFFFFFF)
        self.k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)

    def word(self, env_ids, episode, t, purpose, j):
        j = np.asarray(j, np.int64)
        ctr3 = (np.uint64(purpose) << np.uint64(24)) | (j // 4).astype(np.uint64)
        out = philox4x32_10(env_ids, episode, t, ctr3, self.k0, self.k1)
        lane = np.broadcast_to(j % 4, np.broadcast(out[0], j).shape)
        return np.choose(lane, out).astype(np.uint64)


def uniform_int(m, w):
    return ((np.asarray(w, np.uint64) * np.asarray(m, np.uint64)) >> np.uint64(32)).astype(np.int64)


def select_bit(mask, r):
    """Index of the r-th (0-based) set bit of each uint64 in `mask` (vectorised)."""
    mask = np.asarray(mask, np.uint64)
    r = np.asarray(r, np.int64).copy()
    out = np.full(np.broadcast(mask, r).shape, -1, np.int64)
    m = np.broadcast_to(mask, out.shape).copy()
    for b in range(64):
        bit = ((m >> np.uint64(b)) & np.uint64(1)).astype(bool)
        hit = bit & (r == 0) & (out < 0)
        out[hit] = b
        r = np.where(bit, r - 1, r)
    return out
