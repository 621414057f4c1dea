"""Per-sweep time of one domain tile vs the halo depth K (SV_DOMAIN_DEPTH: sweeps per exchange), on one GPU:
a 1x1 tile with its halos through RCCL to itself (the RCCL code path) and without RCCL, at the config-4 tile
sizes (L=4096 on 1, 2, 8 GPUs: 4096^2, 4096x2048, 2048x1024).
  python scripts/perf/deep_halo.py [depths ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, ghost_frame, unique_id  # noqa: E402

depths = sys.argv[1:] or ['1', '2', '4', '8']
for Nt, Nx in ([tuple(int(v) for v in os.environ['SV_SIZES'].split('x'))] if os.environ.get('SV_SIZES') else
               [(2048, 1024), (4096, 2048), (4096, 4096)]):
    for loop in (True, False):
        for K in depths:
            os.environ['SV_DOMAIN_DEPTH'] = K
            kw = dict(unique_id=unique_id()) if loop else {}
            dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1, **kw)
            dom.cold()
            g = np.random.default_rng(0)
            dom.run(64, g)
            n = 256
            t0 = time.perf_counter()
            st = dom.run(n, g)
            t1 = time.perf_counter()
            print(f'{Nt}x{Nx} rccl={int(loop)} K={K} frame={ghost_frame(Nt, Nx, (1, 1))}: '
                  f'{(t1 - t0) / n * 1e6:.1f} us/sweep, rejections {sum(s.rejections for s in st)}', flush=True)
            dom.close()
