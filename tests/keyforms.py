"""The action dicts of the keys_* fixtures (tests/golden/make_golden.py:run_keys): per step, entries
in recorded order, each keyed in form 0 str(a), 1 int a, 2 str(a - n), 3 int(a - n)."""


def key_dict(form, agent, act, n):
    d = {}
    for f, a, v in zip(form, agent, act):
        if f < 0:
            break
        d[[str(int(a)), int(a), str(int(a) - n), int(a) - n][int(f)]] = int(v)
    return d


def encoded_order(d, n, width):
    """The dict as wh_step/wh_vector_step order entries: agent | (action % 9 + 1) << 8, -1 padded."""
    out = [-1] * width
    for s, (k, v) in enumerate(d.items()):
        idx = int(k)
        out[s] = (idx + n if idx < 0 else idx) | ((int(v) % 9 + 1) << 8)
    return out
