"""Phase-ablation timing of the fused step kernel (timing only: results are wrong by design).
Needs the ablation build: bash tools/build_variant.sh ablation -DWH_ABLATION, then run with
WAREHOUSE_AMD_LIB=build_ab/ablation.so (the production library compiles the ablation switches out).
WH_ABLATE bits: 1 policy, 2 move, 4 expiry, 8 pickup, 16 regeneration, 32 delivery, 64 reward/done
stores, 128 auto-reset.  ABL_STAGGER=1: desynchronised episodes (BatchedWarehouse.stagger).
The library comes from WAREHOUSE_AMD_LIB."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rllib-warehouse_amd")]
import torch  # noqa: E402
import warehouse  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "medium"
na = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B, C = 65536, 200
env = warehouse.BatchedWarehouse(variant, B, na, seed=1)
rew = torch.zeros((C, B, na), device="cuda")
dn = torch.zeros((C, B), dtype=torch.uint8, device="cuda")
masks = [int(m) for m in os.environ.get("ABL_MASKS", "0,1,2,4,8,16,32,17,63,64,128,127,255").split(",")]
res = {m: [] for m in masks}
STAGGER = os.environ.get("ABL_STAGGER") == "1"   # desynchronised episodes (bench.py's desync leg)
for rnd in range(5):
    for m in masks:
        os.environ["WH_ABLATE"] = "0"
        env.reset()
        if STAGGER:
            import numpy as np

            env.stagger((np.arange(B, dtype=np.int64) * 37) % int(env.geometry["T"]))
        os.environ["WH_ABLATE"] = str(m)
        env.rollout(C, "greedy", 0.0, rewards=rew, dones=dn)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout(C, "greedy", 0.0, rewards=rew, dones=dn)
        torch.cuda.synchronize()
        res[m].append((time.perf_counter() - t0) / C * 1e6)
os.environ["WH_ABLATE"] = "0"
for m in masks:
    v = sorted(res[m])
    print(f"ablate={m:2d} us/step median={v[len(v)//2]:.3f} min={v[0]:.3f}")
