"""The dict sampler route (WarehouseBaseEnv: poll -> send_actions -> try_reset of finished envs),
the loop RLlib's sampler runs over a BaseEnv (scripts/train.py:29-43), timed wall-clock.  Random
actions drawn on the host; staggered episodes arise from try_reset only being called for finished
envs.  Prints one JSON line.  WH_PKG_DIR selects another package copy for same-box A/B runs."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("WH_PKG_DIR", os.path.join(ROOT, "rllib-warehouse_amd"))]
import numpy as np  # noqa: E402
from warehouse.vector import WarehouseBaseEnv  # noqa: E402

B = int(os.environ.get("BE_ENVS", "256"))
STEPS = int(os.environ.get("BE_STEPS", "400"))
variant = os.environ.get("BE_VARIANT", "small")
rng = np.random.default_rng(0)
be = WarehouseBaseEnv(variant, B, train=True, seed=0)


def loop(steps):
    agent_steps = resets = 0
    for _ in range(steps):
        obs, rew, dones, _, _ = be.poll()
        acts = {}
        for e, od in obs.items():
            if dones.get(e, {}).get("__all__", False):
                od = be.try_reset(e)          # its first observation: act on it this round
                resets += 1
            acts[e] = {a: int(rng.integers(9)) for a in od}
            agent_steps += len(od)
        be.send_actions(acts)
    return agent_steps, resets


loop(20)
t0 = time.perf_counter()
n, r = loop(STEPS)
dt = time.perf_counter() - t0
print(json.dumps({"route": f"WarehouseBaseEnv {variant} Train, B={B}, random actions, {STEPS} poll/send rounds",
                  "agent_steps": n, "try_resets": r, "wall_s": dt, "agent_steps_per_s": n / dt,
                  "ms_per_round": 1e3 * dt / STEPS}), flush=True)
