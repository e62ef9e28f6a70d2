"""Variant geometry table (warehouse/variants.py:19-62 of the reference) as data."""

GEOMETRY = {
    # name: area_dimension D, num_requests R, pickup_racks_arrangement, episode_duration T,
    #       pickup_wait_duration W, max_num_agents
    "small": dict(D=12, R=4, racks=(4, 8), T=200, W=200, max_agents=4),     # variants.py:19-32
    "medium": dict(D=16, R=9, racks=(4, 8, 12), T=200, W=200, max_agents=9),  # variants.py:35-47
    "large": dict(D=20, R=16, racks=(4, 8, 12, 16), T=200, W=200, max_agents=16),  # variants.py:50-62
}


def pickup_cells(D, racks):
    """Pickup point table in the reference's order (core.py:170-175)."""
    out = []
    for x in racks:
        for y in racks:
            out.extend([(x - 1, y - 1), (x, y - 1), (x - 1, y), (x, y)])
    return out


def delivery_cells(D):
    """Delivery point table in the reference's order (core.py:177-188)."""
    out = []
    for v in range(2, D - 2):
        out.extend([(v, 0), (0, v), (v, D - 1), (D - 1, v)])
    return out
