"""Assert-mode kernels (-DWH_CHECK, build_ab/check.so built by __graft_entry__.build()): SURVEY §5's
invariants checked inside the kernels after every state load, step and reset -- exactly R open
requests (core.py:210-221, 338-351), live agents inside the grid, carried targets on delivery
cells (core.py:177-188), request bytes valid delivery indices, open mask == table, n <= slots.

The check library is loaded in a child process (a process loads one libwarehouse_amd), which runs
fused rollouts across episode ends for every variant, a Train variant (per-episode n), the sampler
step with masks and the fuzzed dense states of test_gpu_fuzz, then reads wh_check_read: zero
violations over millions of checked env-states.  A positive control (a state with R+1 open
requests) must trip the checker.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_LIB = os.path.join(ROOT, "build_ab", "check.so")

CHILD = r"""
import ctypes, json, sys
import numpy as np
sys.path[:0] = [ROOT, ROOT + "/rllib-warehouse_amd"]
import torch
import warehouse
from warehouse import _native as nat
lib = nat.lib()
assert b"assert mode" in lib.wh_version(), lib.wh_version()
assert nat.version_sha(lib.wh_version()) == nat.tree_source_sha(), "stale check.so"
out = (ctypes.c_uint64 * 4)()
def read(clear=1):
    assert lib.wh_check_read(out, clear) == 0
    return [int(v) for v in out]
read()
res = {}
for variant, na, B, steps in (("small", 4, 8192, 450), ("medium", 8, 65536, 450), ("large", 16, 16384, 420),
                              ("medium", 2, 4096, 250), ("large", 8, 4096, 250)):
    env = warehouse.BatchedWarehouse(variant, B, na, seed=3)
    env.reset()
    rew = torch.zeros((steps, B, na), device="cuda")
    dn = torch.zeros((steps, B), dtype=torch.uint8, device="cuda")
    env.rollout(steps, "greedy", 0.0, rewards=rew, dones=dn)    # fused fast path
    env.rollout(steps, "greedy", 0.3)                            # generic path, coin on
    res[f"{variant}{na}"] = read()
env = warehouse.BatchedWarehouse("medium", 32768, train=True, seed=8)
env.reset()
env.rollout(430, "greedy", 0.1)
res["medium_train"] = read()
env = warehouse.BatchedWarehouse("large", 8192, 16, seed=5)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for s in range(60):
    acts = torch.randint(0, 9, (8192, 16), device="cuda", dtype=torch.int32, generator=g)
    mask = torch.rand(8192, device="cuda", generator=g) < 0.7
    env.vector_step(acts, autoreset=True, observe=(s % 10 == 0), mask=mask)
res["vector_step"] = read()
# positive control: R + 1 open requests
B = 256
env = warehouse.BatchedWarehouse("medium", B, 1, seed=1)
P, R = env.P, env.R
pk = np.full((B, P), -1, np.int32); pk[:, : R + 1] = np.arange(R + 1)
env.from_canonical(dict(pos=np.ones((B, 1, 2), np.int32), agent_target=np.full((B, 1), -1, np.int32),
                        pickup_target=pk, pickup_timer=np.where(pk > -1, 50, -1).astype(np.int32),
                        t=np.full(B, 3, np.int32), n=np.ones(B, np.int32)))
env.step(np.full((B, 1), 4, np.int32))
res["control"] = read()
print("CHECK_RESULT " + json.dumps(res))
"""


def test_assert_mode_kernels_find_no_violation():
    assert os.path.exists(CHECK_LIB), "build_ab/check.so missing: run __graft_entry__.build()"
    env = dict(os.environ, WAREHOUSE_AMD_LIB=CHECK_LIB)
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + CHILD], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("CHECK_RESULT ")][-1]
    res = json.loads(line[len("CHECK_RESULT "):])
    for name, (viol, env_id, code, checked) in res.items():
        if name == "control":
            continue
        assert viol == 0, f"{name}: {viol} violations, first env {env_id}, checks failed {code:#x}"
        assert checked > 0
    viol, _, code, _ = res["control"]
    assert viol > 0 and code & 2, res["control"]           # "exactly R open requests" tripped
