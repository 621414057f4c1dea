"""One periodic Nt x Nx domain tile (no RCCL) for a traced run: 64 warm sweeps, then `sweeps` timed ones.
Usage: domain_trace.py Nt Nx sweeps"""
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain  # noqa: E402

Nt, Nx, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
d = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1)
d.cold()
g = np.random.default_rng(0)
d.run(64, g)
t0 = time.perf_counter()
st = d.run(n, g)
t1 = time.perf_counter()
print(f'{Nt}x{Nx}: {(t1 - t0) / n * 1e6:.1f} us/sweep wall, rejections {sum(s.rejections for s in st)}', flush=True)
d.close()
