"""Per-wave timeline of one fused-rollout launch from a -DWH_TIMING build (s_memrealtime, 100 MHz):
entry, tables in LDS (after the workgroup barrier), state in registers and LDS (the loop starts),
step loop done, state stores drained.  Shows where a short launch's fixed cost goes.
    bash tools/build_variant.sh timing -DWH_TIMING
    WAREHOUSE_AMD_LIB=build_ab/timing.so python tools/launch_timeline.py
"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]
SLOTS = 6


def main():
    import numpy as np
    import torch

    import warehouse

    lib = ctypes.CDLL(os.environ["WAREHOUSE_AMD_LIB"])
    lib.wh_debug_times.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    dev = torch.device("cuda", 0)
    for variant, na in (("medium", 8), ("large", 16)):
        B = 65536
        W = B // 64
        env = warehouse.BatchedWarehouse(variant, B, na, seed=3, device=dev)
        env.reset()
        T = int(env.geometry["T"])
        rew = torch.zeros((40, B, na), device=dev)
        dn = torch.zeros((40, B), dtype=torch.uint8, device=dev)
        t = 0

        def run(k):
            nonlocal t
            env.rollout(k, "greedy", 0.0, rewards=rew[:k], dones=dn[:k])
            torch.cuda.synchronize()
            t = (t + k) % T

        def goto(target):
            while (target - t) % T:
                run(min((target - t) % T, 40))

        buf = (ctypes.c_uint64 * (W * SLOTS))()
        for lab, start, k in (("mid_k1", 20, 1), ("mid_k20", 20, 20), ("cross_k20", T - 10, 20)):
            rows = []
            for _ in range(5):
                goto(start)
                run(k)
                assert lib.wh_debug_times(buf, W * SLOTS) == 0
                a = np.frombuffer(buf, dtype=np.uint64).reshape(W, SLOTS)[:, :5].astype(np.int64)
                rows.append(a)
            spans = []
            for a in rows:
                t0 = a[:, 0].min()
                spans.append(dict(span=(a[:, 4].max() - t0) * 10, entry_skew=(a[:, 0].max() - t0) * 10,
                                  tables=np.median(a[:, 1] - a[:, 0]) * 10, state=np.median(a[:, 2] - a[:, 1]) * 10,
                                  loop=np.median(a[:, 3] - a[:, 2]) * 10, loop_max=(a[:, 3] - a[:, 2]).max() * 10,
                                  store=np.median(a[:, 4] - a[:, 3]) * 10,
                                  last_loop_end=(a[:, 3].max() - t0) * 10))
            med = {key: statistics.median(s[key] for s in spans) for key in spans[0]}
            print(f"{variant}-{na} {lab:10s} " + " ".join(f"{key}={v / 1000:.2f}us" for key, v in med.items()),
                  flush=True)


if __name__ == "__main__":
    main()
