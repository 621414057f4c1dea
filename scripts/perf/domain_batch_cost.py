"""Per-sweep time of a 2048x1024 tile through RCCL loopback vs the batch size (SV_DOMAIN_BATCH), with and without
rejection prediction: what a batch (all-gather, synchronization, planning) and an abort cost on one GPU."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, unique_id  # noqa: E402

Nt, Nx = 2048, 1024
for pred in ('0', '1'):
    for B in ('4', '8', '16', '32', '64'):
        os.environ['SV_DOMAIN_PREDICT'] = pred
        os.environ['SV_DOMAIN_BATCH'] = B
        dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1, unique_id=unique_id())
        dom.cold()
        g = np.random.default_rng(0)
        dom.run(64, g)
        n = 512
        t0 = time.perf_counter()
        st = dom.run(n, g)
        t1 = time.perf_counter()
        print(f'predict={pred} batch={B}: {(t1 - t0) / n * 1e6:.1f} us/sweep, rejections {sum(s.rejections for s in st)}',
              flush=True)
        dom.close()
