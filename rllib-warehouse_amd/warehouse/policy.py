"""The SAC policy network on the device (wh_mlp_forward): `trainer.compute_action(obs)` of
scripts/rollout.py:72 for every agent row of a batch, so a trained-policy rollout stays on the
GPU next to the simulator.

Architecture = the policy_model of scripts/experiments/warehouse-{small,medium,large}-sac/*.yaml:
flat observation row (9R+1) -> Linear -> ReLU -> Linear -> ReLU -> Linear -> 9 action logits, hidden
sizes [256,256] / [512,512] / [1024,256].  Weights come in torch nn.Linear layout ([out, in]); no
checkpoint ships with the reference, so `MLPPolicy(variant)` initialises them like nn.Linear's
default (U(-1/sqrt(fan_in), 1/sqrt(fan_in))) from a seed.

precision="bf16" (default, fast): bf16 MFMA, f32 accumulation, activations rounded to bf16 between
layers.  precision="f32": exact f32 on v_mfma_f32_32x32x2_f32 (an fmaf chain per output), i.e. the
reference's TF fp32 policy up to summation order -- about 6x slower.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _native as nat
from ._geometry import GEOMETRY
from .batched import require_device

HIDDEN = {"small": (256, 256), "medium": (512, 512), "large": (1024, 256)}
NUM_ACTIONS = 9
PRECISIONS = {"bf16": nat.WH_MLP_BF16, "f32": nat.WH_MLP_F32}


def init_weights(in_dim: int, hidden0: int, hidden1: int, seed: int = 0) -> Dict[str, np.ndarray]:
    """nn.Linear-style uniform init, float32, [out, in] layout."""
    rng = np.random.RandomState(seed)
    out = {}
    for name, (fo, fi) in (("0", (hidden0, in_dim)), ("1", (hidden1, hidden0)), ("2", (NUM_ACTIONS, hidden1))):
        bound = 1.0 / np.sqrt(fi)
        out["w" + name] = rng.uniform(-bound, bound, size=(fo, fi)).astype(np.float32)
        out["b" + name] = rng.uniform(-bound, bound, size=(fo,)).astype(np.float32)
    return out


class MLPPolicy:
    def __init__(self, variant: str = "medium", weights: Optional[Dict[str, object]] = None, *,
                 seed: int = 0, device=None, precision: str = "bf16"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        R = GEOMETRY[variant]["R"]
        self.in_dim = 9 * R + 1
        self.hidden = HIDDEN[variant]
        self.precision = precision
        self.device = require_device(device)
        self.desc = nat.WhMlpDesc(self.in_dim, self.hidden[0], self.hidden[1], NUM_ACTIONS, PRECISIONS[precision])
        nbytes = ctypes.c_int64()
        nat.check(nat.lib().wh_mlp_query(ctypes.byref(self.desc), ctypes.byref(nbytes)), "wh_mlp_query")
        if weights is None:
            weights = init_weights(self.in_dim, *self.hidden, seed=seed)
        self.weights = {k: np.ascontiguousarray(np.asarray(v.cpu() if torch.is_tensor(v) else v, np.float32))
                        for k, v in weights.items()}
        w = self.weights
        shapes = dict(w0=(self.hidden[0], self.in_dim), b0=(self.hidden[0],), w1=(self.hidden[1], self.hidden[0]),
                      b1=(self.hidden[1],), w2=(NUM_ACTIONS, self.hidden[1]), b2=(NUM_ACTIONS,))
        for k, shp in shapes.items():
            if w[k].shape != shp:
                raise ValueError(f"{k}: expected {shp}, got {w[k].shape}")
        self.packed = torch.empty(int(nbytes.value), dtype=torch.uint8, device=self.device)
        fp = ctypes.POINTER(ctypes.c_float)
        args = [w[k].ctypes.data_as(fp) for k in ("w0", "b0", "w1", "b1", "w2", "b2")]
        with torch.cuda.device(self.device):
            nat.check(nat.lib().wh_mlp_pack(ctypes.byref(self.desc), *args, self.packed.data_ptr()), "wh_mlp_pack")
        self._step = 0

    def forward(self, obs: torch.Tensor, *, explore: bool = False, seed: int = 0, step: Optional[int] = None,
                actions: Optional[torch.Tensor] = None, logits: Optional[torch.Tensor] = None):
        """obs [..., 9R+1] f32 device rows -> (actions [...] int32, logits [..., 9] f32 or None).
        `logits` / `actions` may be passed as output buffers; pass logits=True for a fresh one."""
        lead = obs.shape[:-1]
        if obs.shape[-1] != self.in_dim or obs.dtype != torch.float32 or not obs.is_contiguous():
            raise ValueError(f"obs must be contiguous float32 [..., {self.in_dim}]")
        rows = int(np.prod(lead)) if lead else 1
        if actions is None:
            actions = torch.empty(lead, dtype=torch.int32, device=self.device)
        if logits is True:
            logits = torch.empty((*lead, NUM_ACTIONS), dtype=torch.float32, device=self.device)
        if step is None:
            step, self._step = self._step, self._step + 1
        nat.check(nat.lib().wh_mlp_forward(ctypes.byref(self.desc), self.packed.data_ptr(), rows, obs.data_ptr(),
                                           nat.ptr(logits if logits is not None and logits is not False else None),
                                           actions.data_ptr(), int(bool(explore)), int(seed), int(step) & 0xFFFFFFFF,
                                           nat.stream_of(self.device)), "wh_mlp_forward")
        return actions, (logits if torch.is_tensor(logits) else None)

    __call__ = forward

    def forward_x(self, xfrag: torch.Tensor, rows: int, *, explore: bool = False, seed: int = 0,
                  step: Optional[int] = None, actions: Optional[torch.Tensor] = None,
                  logits: Optional[torch.Tensor] = None):
        """forward() on BatchedWarehouse.observe_x()'s fragment-order operand (rows = B x NA agent
        rows; bf16 precision only): the same actions/logits as forward() on the f32 rows."""
        if self.precision != "bf16":
            raise ValueError("forward_x needs precision='bf16'")
        if actions is None:
            actions = torch.empty(rows, dtype=torch.int32, device=self.device)
        if logits is True:
            logits = torch.empty((rows, NUM_ACTIONS), dtype=torch.float32, device=self.device)
        if step is None:
            step, self._step = self._step, self._step + 1
        nat.check(nat.lib().wh_mlp_forward_x(ctypes.byref(self.desc), self.packed.data_ptr(), int(rows),
                                             xfrag.data_ptr(),
                                             nat.ptr(logits if logits is not None and logits is not False else None),
                                             actions.data_ptr(), int(bool(explore)), int(seed), int(step) & 0xFFFFFFFF,
                                             nat.stream_of(self.device)), "wh_mlp_forward_x")
        return actions, (logits if torch.is_tensor(logits) else None)


def policy_rollout(env, net: MLPPolicy, steps: int, *, explore: bool = False, seed: int = 0,
                   first_step: int = 0, record=None, operand: str = "auto"):
    """scripts/rollout.py's loop (compute_action per agent -> env.step, until done) for every env
    of a BatchedWarehouse, on the device: per step one network forward over all B x NA observation
    rows, then the step (step + auto-reset + the next rows).  operand="fragments" (the default for
    bf16 networks) hands the rows to the network as its layer-0 operand (wh_vector_step_x writes
    it, wh_mlp_forward_x reads it: the same actions, no f32 rows materialised); "rows" uses the
    float32 observation rows (wh_vector_step).  `record`, if given, is called as record(step, actions, rewards,
    dones) with env-owned device tensors.  Returns the last step's observations (the fragment
    buffer or the obs tensor)."""
    if operand == "auto":
        operand = "fragments" if net.precision == "bf16" else "rows"
    if operand not in ("fragments", "rows"):
        raise ValueError("operand must be 'auto', 'fragments' or 'rows'")
    B, NA = env.B, env.agent_slots
    acts = torch.empty((B, NA), dtype=torch.int32, device=env.device)
    frag = operand == "fragments"
    obs = env.observe_x() if frag else env.observe()
    for s in range(steps):
        if frag:
            net.forward_x(obs, B * NA, explore=explore, seed=seed, step=first_step + s, actions=acts.view(-1))
            obs, rew, done = env.vector_step_x(acts, autoreset=True)   # step + the next operand
        else:
            net(obs.view(B * NA, -1), explore=explore, seed=seed, step=first_step + s, actions=acts.view(-1))
            obs, rew, done = env.vector_step(acts, autoreset=True, observe=True)
        if record is not None:
            record(s, acts, rew, done)
    return obs
