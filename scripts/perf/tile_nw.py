"""Per-sweep wall time of one periodic domain tile (no RCCL) under the current environment (SV_DOMAIN_NW,
SV_DOMAIN_TH16, SV_DOMAIN_TH8, ...).  python scripts/perf/tile_nw.py TAG [Nt Nx]"""
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain  # noqa: E402

tag = sys.argv[1]
Nt, Nx = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (2048, 1024)
warm = VillainDomain(2048, 2048, (1, 1), kappa=0.5, W=1)  # clocks to steady state before the timing
warm.cold()
warm.run(1500, np.random.default_rng(9))
warm.close()
dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1)
dom.cold()
g = np.random.default_rng(0)
dom.run(64, g)
best = []
for rep in range(3):
    n = 512
    t0 = time.perf_counter()
    st = dom.run(n, g)
    t1 = time.perf_counter()
    best.append((t1 - t0) / n * 1e6)
print(f'{tag} {Nt}x{Nx}: ' + ' '.join(f'{b:.1f}' for b in best) + ' us/sweep', flush=True)
dom.close()
