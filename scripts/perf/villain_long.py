"""Long thinned Villain chains at one (N, kappa): the NeighborhoodUpdate alone (counter-based, and PCG64) kept every
`stride` sweeps, against the reference's Link + Site + Exact + Cohomology suite; ActionDensity and WindingSquared
means with blocked-bootstrap errors.  Usage: villain_long.py N kappa configs stride"""
import sys

import numpy as np

sys.path.insert(0, '.')
import supervillain_amd as sv  # noqa: E402
from supervillain_amd.generator import KeepEvery, Sequentially  # noqa: E402
from supervillain_amd.generator import villain as V  # noqa: E402
from tests.statparity import blocked_bootstrap  # noqa: E402
from tests.test_gpu_statparity import villain_observables  # noqa: E402

N, kappa, steps, stride = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
L = sv.Lattice2D(N)
S = sv.Villain(L, kappa, 1)
for name in ('philox', 'pcg64-nbhd', 'suite'):
    if name == 'philox':
        g = KeepEvery(stride, V.NeighborhoodUpdate(S, philox=0x5EED0009))
    elif name == 'pcg64-nbhd':
        h = V.NeighborhoodUpdate(S)
        h.rng = np.random.default_rng(9)
        g = KeepEvery(stride, h)
    else:
        gens = [V.LinkUpdate(S), V.SiteUpdate(S), V.ExactUpdate(S), V.CohomologyUpdate(S)]
        for i, x in enumerate(gens):
            x.rng = np.random.default_rng(90 + i)
        g = Sequentially(gens)
    E = sv.Ensemble(S).generate(steps, g)
    o = villain_observables(np.asarray(E.configuration.phi.array), np.asarray(E.configuration.n.array), kappa)
    cut = steps // 10
    a, ea = blocked_bootstrap(o[cut:, 0], 100)
    w, ew = blocked_bootstrap(o[cut:, 3], 100)
    print(f'N={N} kappa={kappa} {name}: ActionDensity {a:.5f} +- {ea:.5f}, WindingSquared {w:.5f} +- {ew:.5f}', flush=True)
