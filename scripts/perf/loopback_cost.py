"""Per-sweep time of a 1x1 domain whose halos go through RCCL to itself (the RCCL code path on one GPU)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, unique_id
L = 4096
for loop in (False, True):
    kw = dict(unique_id=unique_id()) if loop else {}
    dom = VillainDomain(L, L, (1, 1), kappa=0.5, W=1, **kw)
    dom.cold()
    g = np.random.default_rng(0)
    dom.run(10, g)
    t0 = time.perf_counter(); st = dom.run(200, g); t1 = time.perf_counter()
    print(f'loopback={loop}: per sweep {(t1-t0)/200*1e6:.1f} us, rejections {sum(s.rejections for s in st)}', flush=True)
    dom.close()
