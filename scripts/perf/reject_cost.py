"""Per-tile sweep time vs tile count (emulated on one GPU) and the rejection replays met."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain
L = 4096
for ty, tx in [(1, 1), (1, 2), (2, 4)]:
    dom = VillainDomain(ty * L, tx * L, (ty, tx), kappa=0.5, W=1)
    dom.cold()
    g = np.random.default_rng(0)
    dom.run(10, g)
    for K in (200,):
        t0 = time.perf_counter(); st = dom.run(K, g); t1 = time.perf_counter()
        rj = sum(s.rejections for s in st)
        per = (t1 - t0) / K / (ty * tx)
        print(f'tiles {ty}x{tx}: {K} sweeps {t1-t0:.3f} s, per tile-sweep {per*1e6:.1f} us, rejections {rj}', flush=True)
    dom.close()
