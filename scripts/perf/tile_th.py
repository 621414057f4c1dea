"""Per-sweep time of one periodic domain tile (no RCCL) vs the strip height SV_FUSED_TH, at the config-4 per-GPU
tile sizes.  python scripts/perf/tile_th.py TH ..."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain  # noqa: E402

sizes = [tuple(int(v) for v in os.environ['SV_SIZES'].split('x')) ] if os.environ.get('SV_SIZES') else [(2048, 1024), (4096, 2048), (4096, 4096)]
warm = VillainDomain(4096, 4096, (1, 1), kappa=0.5, W=1)  # clocks to steady state before the first timing
warm.cold()
warm.run(2000, np.random.default_rng(9))
warm.close()
for Nt, Nx in sizes:
    for th in sys.argv[1:] or ['']:
        if th:
            os.environ['SV_FUSED_TH'] = th
        else:
            os.environ.pop('SV_FUSED_TH', None)
        dom = VillainDomain(Nt, Nx, (1, 1), kappa=0.5, W=1)
        dom.cold()
        g = np.random.default_rng(0)
        dom.run(64, g)
        n = 256
        t0 = time.perf_counter()
        dom.run(n, g)
        t1 = time.perf_counter()
        print(f'{Nt}x{Nx} TH={th or "auto"}: {(t1 - t0) / n * 1e6:.1f} us/sweep', flush=True)
        dom.close()
