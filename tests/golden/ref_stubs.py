"""Minimal stand-ins for `gym` and `ray` so the read-only reference package imports here.

Golden-generation infrastructure only (used by `make_golden.py` in the build container, where
`/root/reference` exists).  Nothing on the GPU box imports this module.

The reference needs, from gym, only the space classes it constructs in
`warehouse/core.py:118-148` (Discrete, Box, MultiBinary, Dict) and their `contains` checks used by
`baseline/run.py:36-37,58-59`; from ray it needs only the `MultiAgentEnv` base class
(`warehouse/core.py:6,73`).  Neither package is installed in this image.
"""
from __future__ import annotations

import sys
import types

import numpy as np


class _Space:
    pass


class _Discrete(_Space):
    def __init__(self, n):
        self.n = int(n)
        # gym's spaces draw from their own generator, never from the global numpy stream
        self._rng = np.random.RandomState(0)

    def sample(self):
        return int(self._rng.randint(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n


class _Box(_Space):
    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))


class _MultiBinary(_Space):
    def __init__(self, n):
        self.n = n

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == (self.n,) and bool(np.all((x == 0) | (x == 1)))


class _Dict(_Space):
    def __init__(self, spaces):
        # gym.spaces.Dict sorts the keys of a plain dict
        self.spaces = dict(sorted(spaces.items()))

    def contains(self, x):
        return all(k in x and s.contains(x[k]) for k, s in self.spaces.items())


def install() -> None:
    """Register the fake modules in sys.modules (idempotent)."""
    if "gym" in sys.modules and getattr(sys.modules["gym"], "_wh_stub", False):
        return
    gym = types.ModuleType("gym")
    gym._wh_stub = True
    spaces = types.ModuleType("gym.spaces")
    spaces.Space, spaces.Discrete, spaces.Box = _Space, _Discrete, _Box
    spaces.MultiBinary, spaces.Dict = _MultiBinary, _Dict
    gym.spaces, gym.Space = spaces, _Space
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces

    for name in ("ray", "ray.rllib", "ray.rllib.env", "ray.rllib.env.multi_agent_env"):
        sys.modules[name] = types.ModuleType(name)

    class MultiAgentEnv:  # noqa: D401 - stand-in base class
        def __init__(self):
            pass

    sys.modules["ray.rllib.env.multi_agent_env"].MultiAgentEnv = MultiAgentEnv


def import_reference(ref_root: str = "/root/reference"):
    """Import the reference `warehouse` package and `baseline/solvers.py` / `baseline/run.py`."""
    install()
    for p in (ref_root + "/baseline", ref_root):
        if p not in sys.path:
            sys.path.insert(0, p)
    import warehouse  # noqa: F401  (the reference package)
    import solvers  # noqa: F401
    import run  # noqa: F401

    return sys.modules["warehouse"], sys.modules["solvers"], sys.modules["run"]
