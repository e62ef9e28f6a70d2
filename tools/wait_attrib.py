"""Per-phase attribution of the fused step kernel's waits and instructions.

Runs fused greedy rollouts on the timing-only ablation build (-DWH_ABLATION: WH_ABLATE bit masks
skip phases, results wrong by design) in a fixed order, so that a rocprofv3 --pmc run of this
script gives every k_step dispatch its phase mask and launch length:

    bash tools/build_variant.sh ablm8 -DWH_ONLY_MEDIUM8 -DWH_ABLATION
    WAREHOUSE_AMD_LIB=$PWD/build_ab/ablm8.so WAREHOUSE_AMD_AB=1 timeout -s KILL 200 rocprofv3 \\
        --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_LDS \\
        SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/wattr -o run -- python3 tools/wait_attrib.py
    python tools/wait_attrib_report.py gpurun_out/wattr

WH_ABLATE bits (tools/ablate.py): 1 policy, 2 move, 4 expiry, 8 pickup, 16 regeneration,
32 delivery, 64 reward/done stores, 128 auto-reset.  K = 1 launches are mostly the fixed part
(prologue: state and table loads, pickup plane, grid clear; epilogue: state stores); the report
separates fixed and per-step parts from K = 1, 20, 200.  Each (K, mask) group is M launches from a
fresh reset (t = 0), the first dropped by the report as warm-up.  The plan is
written to gpurun_out/wattr_plan.json.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def main():
    variant = os.environ.get("WATTR_VARIANT", "medium")
    na = int(os.environ.get("WATTR_AGENTS", "8"))
    masks = [int(m) for m in os.environ.get("WATTR_MASKS", "0,1,2,8,16,32,64,128,255").split(",")]
    Ks = [int(k) for k in os.environ.get("WATTR_STEPS", "1,20,200").split(",")]
    M = 4
    B = 65536
    env = warehouse.BatchedWarehouse(variant, B, na, seed=1)
    rew = torch.zeros((max(Ks), B, na), device="cuda")
    dn = torch.zeros((max(Ks), B), dtype=torch.uint8, device="cuda")
    plan = []
    for K in Ks:
        for m in masks:
            os.environ["WH_ABLATE"] = "0"
            env.reset()
            torch.cuda.synchronize()
            os.environ["WH_ABLATE"] = str(m)
            for _ in range(M):
                env.rollout(K, "greedy", 0.0, rewards=rew[:K], dones=dn[:K])
            torch.cuda.synchronize()
            plan.append({"K": K, "mask": m, "launches": M})
            print(f"K={K} mask={m} done", flush=True)
    os.environ["WH_ABLATE"] = "0"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"variant": variant, "agents": na, "B": B, "plan": plan},
              open(os.path.join(ROOT, "gpurun_out", "wattr_plan.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
