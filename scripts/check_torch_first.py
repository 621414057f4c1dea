"""Load order check for the multi-GPU bench: torch (and its bundled HIP runtime / RCCL) imported
BEFORE libsvhip.so, as bench.py does for N > 1.  Runs a small decomposed chain against the oracle."""
import os
import sys

import torch  # noqa: F401  (must come first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from oracle import oracle as O
from supervillain_amd.domain import VillainDomain, unique_id

N = 64
r = np.random.default_rng(1)
phi0, n0 = r.uniform(-3, 3, (N, N)), r.integers(-2, 3, (2, N, N)).astype(np.int64)
for tiles, uid in [((2, 2), None), ((1, 1), unique_id())]:  # local tiles; RCCL loopback (torch's librccl)
    dom = VillainDomain(N, N, tiles, 0.5, 1, unique_id=uid)
    dom.upload(phi0, n0)
    g1 = np.random.default_rng(3)
    dom.run(4, g1)
    phi, n = dom.download()
    dom.close()
    p, m = phi0.copy(), n0.copy()
    g2 = np.random.default_rng(3)
    O.villain_neighborhood(N, 0.5, 1, p, m, 4, g2)
    assert (phi == p).all() and (n == m).all() and g1.bit_generator.state == g2.bit_generator.state, tiles
print('torch-first load order OK:', torch.__version__)
