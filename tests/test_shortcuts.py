"""The exact node shortcuts of the SC kernel (sc_kernel.hip) against a direct recursive min-sum SC.

Each rule must equal what the reference recursion (polar_sc.py:54-98, min-sum f :46) computes on
the node, whenever the rule's precondition holds: rate-1 (no zero LLR), repetition (always),
SPC (no zero LLR; for odd parity a unique min |alpha| below the +-30 clip).  Inputs include
rounded values (ties, zeros) and saturating magnitudes.
"""
import numpy as np


def _f(x, y):
    xc, yc = np.clip(x, -30, 30), np.clip(y, -30, 30)
    return (np.sign(xc) * np.sign(yc) * np.minimum(np.abs(xc), np.abs(yc))).astype(np.float32)


def _sc(alpha, frozen):
    m = len(alpha)
    if m == 1:
        return np.array([0 if frozen[0] else (0 if alpha[0] > 0 else 1)])
    h = m // 2
    bl = _sc(_f(alpha[:h], alpha[h:]), frozen[:h])
    y = ((1 - 2 * bl).astype(np.float32) * alpha[:h] + alpha[h:]).astype(np.float32)
    br = _sc(y, frozen[h:])
    return np.concatenate([bl ^ br, br])


def test_shortcut_rules_match_recursive_sc():
    rng = np.random.default_rng(1)
    used = {"R1": 0, "REP": 0, "SPC": 0, "SPC_fallback": 0}
    for _ in range(6000):
        m = int(rng.choice([2, 4, 8, 16, 32]))
        al = (rng.standard_normal(m) * rng.choice([0.5, 3, 20, 60])).astype(np.float32)
        if rng.random() < 0.3:
            al = np.round(al).astype(np.float32)
        hd = (al <= 0).astype(int)
        if not (al == 0).any():  # rate-1
            assert np.array_equal(_sc(al, np.zeros(m, bool)), hd)
            used["R1"] += 1
        fz = np.ones(m, bool)
        fz[-1] = False  # repetition: pairwise sum in g order
        y = al.copy()
        while len(y) > 1:
            y = (y[: len(y) // 2] + y[len(y) // 2:]).astype(np.float32)
        assert np.array_equal(_sc(al, fz), np.full(m, 0 if y[0] > 0 else 1))
        used["REP"] += 1
        if (al == 0).any():
            continue
        fz = np.zeros(m, bool)
        fz[0] = True  # SPC (Wagner)
        w = hd.copy()
        if w.sum() % 2:
            a = np.abs(al)
            if (a == a.min()).sum() != 1 or not a.min() < 30:
                used["SPC_fallback"] += 1
                continue
            w[np.argmin(a)] ^= 1
        assert np.array_equal(_sc(al, fz), w)
        used["SPC"] += 1
    assert min(used.values()) > 50, used
