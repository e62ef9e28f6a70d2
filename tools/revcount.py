"""How often the fused rollout's move loop takes the reverse-key variant (waves with co-located
agents) -- run against a -DWH_COUNT_REV build:
    bash tools/build_variant.sh revcount -DWH_COUNT_REV
    WAREHOUSE_AMD_LIB=build_ab/revcount.so python tools/revcount.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]


def main():
    import numpy as np
    import torch

    import warehouse
    from warehouse import _native

    dev = torch.device("cuda", 0)
    L = _native.lib()
    out = (ctypes.c_uint64 * 4)()

    def read():
        assert L.wh_check_read(out, 1) == 0
        return int(out[0]), int(out[1])

    for variant, na in (("medium", 8), ("large", 16)):
        for stagger in (False, True):
            env = warehouse.BatchedWarehouse(variant, 65536, na, seed=3, device=dev)
            env.reset()
            T = int(env.geometry["T"])
            if stagger:
                env.stagger((np.arange(65536, dtype=np.int64) * 37) % T)
            rew = torch.zeros((100, 65536, na), device=dev)
            dn = torch.zeros((100, 65536), dtype=torch.uint8, device=dev)
            env.rollout(20, "greedy", 0.0, rewards=rew[:20], dones=dn[:20])   # the fast instance
            torch.cuda.synchronize()
            read()
            for _ in range(4):
                env.rollout(100, "greedy", 0.0, rewards=rew, dones=dn)
            rev, norev = read()
            print(f"{variant}-{na} stagger={stagger}: reverse-key loops {rev}, crossing-only {norev}, "
                  f"reverse share {rev / max(1, rev + norev):.4f}", flush=True)


if __name__ == "__main__":
    main()
