import numpy as np, sys
sys.path.insert(0, '.')
import supervillain_amd as sv
from oracle import oracle as O
from tests.golden import cases, generator_from, state_of
for c in [c for c in cases('villain_generators.npz') if c['kind'] == 'CohomologyUpdate'][:3]:
    N = c['N']
    S = sv.Villain(sv.Lattice2D(N), c['kappa'], c['W'])
    G = sv.generator.villain.CohomologyUpdate(S)
    G.rng = generator_from(c['rng0'])
    g = generator_from(c['rng0'])
    cfg = {'phi': sv.Form(c['phi0'].reshape(1, N, N).copy(), degree=0, lattice=S.Lattice),
           'n': sv.Form(c['n0'].reshape(2, N, N).copy(), degree=1, lattice=S.Lattice)}
    phi, n = c['phi0'].reshape(N, N).copy(), c['n0'].reshape(2, N, N).copy()
    for k in range(c['sweeps']):
        cfg = G.step(cfg)
        O.villain_generator('CohomologyUpdate', N, c['kappa'], c['W'], phi, n, 1, g)
        a, b = state_of(G.rng), state_of(g)
        print(k, (a == b).all(), a, b, (np.asarray(cfg['n']) == n).all())
