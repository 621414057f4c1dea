"""Per-sweep time of the config-4 N = 8 tile (2048 x 1024) through RCCL loopback by halo depth (SV_DOMAIN_DEPTH: sweeps
per exchange), with rejection prediction on as 8 ranks run it; interleaved repetitions.

    python scripts/perf/domain_depth_cost.py [reps=2] [depths=4,6,8]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, unique_id  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
depths = sys.argv[2].split(',') if len(sys.argv) > 2 else ['4', '6', '8']
Nt, Nx = 2048, 1024
os.environ['SV_DOMAIN_PREDICT'] = '1'
for r in range(reps):
    for K in depths:
        os.environ['SV_DOMAIN_DEPTH'] = K
        dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1, unique_id=unique_id())
        dom.cold()
        g = np.random.default_rng(0)
        dom.run(64, g)
        n = 512
        t0 = time.perf_counter()
        st = dom.run(n, g)
        t1 = time.perf_counter()
        print(f'depth={K} rep {r}: {(t1 - t0) / n * 1e6:.2f} us/sweep, rejections {sum(s.rejections for s in st)}',
              flush=True)
        dom.close()
