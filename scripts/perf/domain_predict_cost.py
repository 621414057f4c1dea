"""Is rejection prediction worth its scan on the strong-scaled ranks?  The config-4 N = 8 tile (2048 x 1024) through
RCCL loopback, with NumPy's Lemire threshold raised so that its own rejections per sweep match what a whole L=4096
lattice meets (every rank aborts on any rank's rejection): interval_n = 6 (13 choices, threshold 9: 9x the rate of the
default 3 choices, 0.018 per sweep of this tile vs 0.0156 for L=4096) -- and at the default interval_n = 1 for
reference; SV_DOMAIN_PREDICT 0 / 1, default batches, 512 sweeps, interleaved repetitions.

    python scripts/perf/domain_predict_cost.py [reps=2]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, unique_id  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
Nt, Nx = 2048, 1024
for r in range(reps):
    for iv in (6, 1):
        for pred in ('0', '1'):
            os.environ['SV_DOMAIN_PREDICT'] = pred
            dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1, interval_n=iv, unique_id=unique_id())
            dom.cold()
            g = np.random.default_rng(0)
            dom.run(64, g)
            n = 512
            t0 = time.perf_counter()
            st = dom.run(n, g)
            t1 = time.perf_counter()
            print(f'interval_n={iv} predict={pred} rep {r}: {(t1 - t0) / n * 1e6:.2f} us/sweep, '
                  f'rejections {sum(s.rejections for s in st)}', flush=True)
            dom.close()
