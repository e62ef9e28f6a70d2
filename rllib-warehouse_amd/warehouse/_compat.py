"""gym / ray imports with minimal stand-ins when they are absent (neither is in this image).

The reference subclasses ray's `MultiAgentEnv` (warehouse/core.py:6,73) and builds gym spaces
(core.py:118-148).  With ray/gym installed the real classes are used, so RLlib sees an ordinary
MultiAgentEnv; without them these stand-ins keep `import warehouse` and the drivers working.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gym is installed
    import gym as _gym

    spaces = _gym.spaces
    HAVE_GYM = True
except ImportError:
    HAVE_GYM = False

    class _Spaces:
        class Space:
            pass

        class Discrete(Space):
            def __init__(self, n):
                self.n = int(n)
                self.np_random = np.random.RandomState(0)   # own generator, like gym's spaces

            def seed(self, seed=None):
                self.np_random = np.random.RandomState(seed)
                return [seed]

            def sample(self):
                return int(self.np_random.randint(self.n))

            def contains(self, x):
                try:
                    return 0 <= int(x) < self.n
                except (TypeError, ValueError):
                    return False

        class Box(Space):
            def __init__(self, low, high, shape, dtype):
                self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

            def contains(self, x):
                x = np.asarray(x)
                if x.shape != self.shape:
                    return False
                if x.size and np.isscalar(self.low) and np.isscalar(self.high):   # two reductions, no temporaries
                    return bool(x.min() >= self.low) and bool(x.max() <= self.high)
                return bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        class MultiBinary(Space):
            def __init__(self, n):
                self.n = n
                self.shape = (n,)

            def contains(self, x):
                x = np.asarray(x)
                if x.shape != (self.n,):
                    return False
                if x.size and x.dtype.kind in "biu":                 # integers: {0, 1} <=> 0 <= x <= 1
                    return bool(x.min() >= 0) and bool(x.max() <= 1)
                return bool(np.all((x == 0) | (x == 1)))

        class Dict(Space):
            def __init__(self, spaces):
                self.spaces = dict(sorted(spaces.items()))

            def contains(self, x):
                return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

            def __getitem__(self, k):
                return self.spaces[k]

    spaces = _Spaces

try:  # pragma: no cover
    from ray.rllib.env.multi_agent_env import MultiAgentEnv
except ImportError:

    class MultiAgentEnv:  # minimal stand-in for ray.rllib.env.multi_agent_env.MultiAgentEnv
        def __init__(self):
            pass

        def render(self, mode="human"):
            raise NotImplementedError
