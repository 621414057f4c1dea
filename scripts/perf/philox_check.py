"""Mean ActionDensity of the Villain NeighborhoodUpdate chain at N=8, kappa=1 (expected near (V-1)/(2V) = 0.492), and
the fraction of consecutive kept configurations that differ: device-resident generation against the per-step loop,
counter-based (Philox) and PCG64 modes."""
import sys

import numpy as np

sys.path.insert(0, '.')
import supervillain_amd as sv  # noqa: E402
from supervillain_amd.generator import villain as V  # noqa: E402
from supervillain_amd.generator import Sequentially  # noqa: E402
from tests.test_gpu_statparity import villain_observables  # noqa: E402

N, kappa, steps = 8, 1.0, int(sys.argv[1]) if len(sys.argv) > 1 else 20000
L = sv.Lattice2D(N)
S = sv.Villain(L, kappa, 1)
for mode in ('philox', 'pcg64'):
    for resident in (True, False):
        g = V.NeighborhoodUpdate(S, philox=0x5EED0001) if mode == 'philox' else V.NeighborhoodUpdate(S)
        if mode == 'pcg64':
            g.rng = np.random.default_rng(7)
        E = sv.Ensemble(S).generate(steps, Sequentially([g]), device_resident=resident)
        phi = np.asarray(E.configuration.phi.array)
        o = villain_observables(phi, np.asarray(E.configuration.n.array), kappa)
        a = o[steps // 10:, 0]
        moved = np.mean(np.any(np.diff(phi, axis=0) != 0, axis=(1, 2, 3)))
        print(f'{mode} resident={resident}: ActionDensity {a.mean():.4f} (halves {a[:len(a)//2].mean():.4f} '
              f'{a[len(a)//2:].mean():.4f}); consecutive configurations differ in {moved:.3f} of steps', flush=True)
