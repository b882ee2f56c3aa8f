"""Code construction: Arikan kernel powers and the reference's RM-weight frozen sets.

Reference: x_run_sn_polar/polar/froze.py:4-16.  The frozen set is the n-k rows of
G = F2^{(x)m} with the smallest weight 2^popcount(i); ties are broken by torch's *unstable* CPU
argsort (froze.py:14), so the exact set depends on the host's sort implementation.  The sets the
reference produced (build container, x86-64 AVX-512) are pinned in data/frozen_sets.npz and
returned by reference_frozen_pos(); get_Kern_frozen_bits() re-runs the reference recipe on
this host, as the reference does.
"""
import math
import os

import numpy as np
import torch as tc

F2 = tc.tensor([[1, 0], [1, 1]], dtype=tc.float32)
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "frozen_sets.npz")
_cache = None


def kron_power(kern, n):
    base = kern.shape[0]
    stages = int(round(math.log(n, base)))
    assert base ** stages == n, f"{n=}, is not power of {base=}"
    m = tc.clone(kern)
    for _ in range(stages - 1):
        m = tc.kron(kern, m)
    return m


def get_Kern_frozen_bits(n, f_num, kern):
    """froze.py:4-16: (G, row weights, frozen_pos) with frozen = the f_num lightest rows."""
    G = kron_power(kern, n)
    w = tc.sum(G, dim=1)
    frozen_pos = tc.sort(tc.argsort(w)[:f_num])[0]
    return G, w, frozen_pos


def reference_frozen_pos(k, n):
    """The frozen positions the reference's froze.py produced for (k, n) (int64 tensor, sorted)."""
    global _cache
    if _cache is None:
        with np.load(_DATA) as d:
            _cache = {key: d[key].astype(np.int64) for key in d.files}
    key = f"k{k}_n{n}"
    if key not in _cache:
        raise KeyError(f"no pinned reference frozen set for (k={k}, n={n}); available: {sorted(_cache)}")
    return tc.from_numpy(_cache[key].copy())


def frozen_mask(frozen_pos, n):
    fp = frozen_pos.cpu().numpy() if isinstance(frozen_pos, tc.Tensor) else np.asarray(frozen_pos)
    m = np.zeros(n, dtype=np.uint8)
    m[fp.astype(np.int64)] = 1
    return m
