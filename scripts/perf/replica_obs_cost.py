"""Config-5 sweep time with and without the inline observables (villain_sweep_hot_fr<OBS>)."""
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd.replicas import VillainReplicas  # noqa: E402

R, N = 1024, 128
for rep in range(2):
    for inline in (True, False):
        B = VillainReplicas(R, N, 0.5, 2)
        B.cold()
        gens = [np.random.default_rng(r) for r in range(R)]
        B.run(64, gens, inline=inline)
        n = 320
        t0 = time.perf_counter()
        B.run(n, gens, inline=inline)
        t1 = time.perf_counter()
        print(f'inline={inline}: {(t1 - t0) / n * 1e6:.1f} us/sweep', flush=True)
        B.close()
