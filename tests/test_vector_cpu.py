"""Host logic of the RLlib-facing adapters (warehouse.vector, warehouse.batched.EpisodeStats):
the flat observation layout against the reference fixtures and the on_episode_end arithmetic."""
import glob
import os

import numpy as np

from oracle import core as oc
from warehouse.batched import custom_metrics_from_bins
from warehouse.vector import OBS_KEYS, flat_observation_space, obs_key_widths, unflatten_row

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_flat_layout_is_sorted_keys_and_covers_golden_rows():
    assert list(OBS_KEYS) == sorted(OBS_KEYS)
    for variant in ("small", "medium", "large"):
        L = oc.layout_for(variant)
        assert sum(obs_key_widths(L.R).values()) == 9 * L.R + 1
        box = flat_observation_space(L.R, L.D)
        for path in sorted(glob.glob(os.path.join(GOLDEN, f"g1_{variant}_*.npz")))[:2]:
            g = np.load(path)
            rows = g["obs"].reshape(-1, g["obs"].shape[-1]).astype(np.float32)
            for row in rows[:: max(1, len(rows) // 50)]:
                assert box.contains(row)
                d = unflatten_row(row, L.R)
                assert list(d) == list(OBS_KEYS)
                np.testing.assert_array_equal(np.concatenate([v.reshape(-1) for v in d.values()]), row)
                assert d["requests"].shape == (L.R, 4) and d["other_positions"].shape == (L.R - 1, 2)


def test_custom_metrics_from_bins_matches_on_episode_end():
    """scripts/train.py:18-23: avg_agent_reward = sum(agent returns) / n per episode."""
    episodes = [(2, 7), (2, 3), (3, 9), (1, 0), (3, 4)]      # (n, episode return summed over agents)
    na = 4
    s = np.zeros(na + 1, np.int64)
    c = np.zeros(na + 1, np.int64)
    mn = np.full(na + 1, 0xFFFFFFFF, np.uint32)
    mx = np.zeros(na + 1, np.uint32)
    for n, r in episodes:
        s[n] += r
        c[n] += 1
        mn[n] = min(mn[n], r)
        mx[n] = max(mx[n], r)
    cm = custom_metrics_from_bins(s, c, mn, mx)
    avgs = [r / n for n, r in episodes]
    a = cm["avg_agent_reward_all"]
    assert abs(a["mean"] - np.mean(avgs)) < 1e-12 and (a["min"], a["max"], a["count"]) == (min(avgs), max(avgs), 5)
    assert cm["avg_agent_reward_2"] == dict(mean=5.0 / 2, min=1.5, max=3.5, count=2)
    assert cm["avg_agent_reward_3"]["mean"] == 13 / 6
    assert "avg_agent_reward_4" not in cm
