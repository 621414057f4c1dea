"""1x1 domain with RCCL loopback halos, 100 sweeps (for rocprofv3)."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain, unique_id
dom = VillainDomain(4096, 4096, (1, 1), kappa=0.5, W=1, unique_id=unique_id())
dom.cold()
g = np.random.default_rng(0)
dom.run(10, g)
t0 = time.perf_counter(); st = dom.run(100, g); t1 = time.perf_counter()
print(f'per sweep {(t1-t0)/100*1e6:.1f} us', flush=True)
dom.close()
