"""Config 1 through the drop-in class: baseline/run.py's loop (greedy solver on the observation
dicts, WarehouseSmall(2), p = 0) with every transition on the GPU.  Prints one JSON line with
episodes, total reward and wall-clock agent-steps/s (host-loop and launch-latency bound: one env)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("WH_PKG_DIR", os.path.join(ROOT, "rllib-warehouse_amd"))]   # A/B: another package copy
import numpy as np  # noqa: E402
import warehouse  # noqa: E402


def greedy(obs, n, p, rng_draw):
    """baseline/solvers.py:27-58 restated on the dicts (drop-in side; the oracle is not used)."""
    acts = {}
    for i in range(n):
        o = obs[str(i)]
        coin = rng_draw()
        if coin < p:
            acts[str(i)] = int(np.random.randint(9))
            continue
        pos = o["self_position"]
        if o["self_availability"][0] == 0:
            tgt = o["self_delivery_target"]
        else:
            req = o["requests"]
            d = np.abs(req[:, 0] - pos[0]) + np.abs(req[:, 1] - pos[1])
            tgt = req[int(np.argmin(d)), :2]
        sx, sy = np.clip(tgt - pos, -1, 1)
        acts[str(i)] = int((sx + 1) * 3 + (sy + 1))
    return acts


EPISODES = int(os.environ.get("C1_EPISODES", "3"))
np.random.seed(0)
env = warehouse.WarehouseSmall(2)
if os.environ.get("C1_WARM"):              # one untimed episode first (launch paths, pinned buffers)
    obs, done = env.reset(), False
    while not done:
        obs, _, dones, _ = env.step(greedy(obs, 2, 0.0, np.random.uniform))
        done = dones["__all__"]
    np.random.seed(0)
t0 = time.perf_counter()
steps, total = 0, 0.0
for ep in range(EPISODES):
    obs = env.reset()
    done = False
    while not done:
        obs, rew, dones, _ = env.step(greedy(obs, 2, 0.0, np.random.uniform))
        total += float(sum(rew.values()))
        steps += 1
        done = dones["__all__"]
dt = time.perf_counter() - t0
print(json.dumps({"config": f"C1: WarehouseSmall(2), greedy p=0, drop-in single env, {EPISODES} episodes"
                            + (" after a warm-up episode" if os.environ.get("C1_WARM") else ""),
                  "episodes": EPISODES, "steps": steps, "total_reward": total,
                  "agent_steps_per_s": 2 * steps / dt, "wall_s": dt}), flush=True)
