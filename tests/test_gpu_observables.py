"""The inline observables on the MI355X against values the REFERENCE measured on its own chains.

tests/golden/villain_observables.npz (tools/make_golden_observables.py) holds, after every NeighborhoodUpdate sweep of
seeded Villain chains (N = 8, 16, 128; W = 1, 2; cold and hot starts), the reference's
ActionDensity (observable/action.py:25-31), InternalEnergyDensity (energy.py:25-30), WindingSquared (winding.py:30-37)
and TorusWrapping (wrapping.py:17-25).  The single-lattice inline reduction (sv_villain_observables, device-resident and
per-step Ensemble paths) and the replica kernels' fused row-store sums (sv_replicas_run, config 5's kernel) must give
those values: floats within 1e-12 relative, the integer wrapping sums exactly."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.replicas import VillainReplicas
from tests.golden import generator_from, observable_groups, observable_start, state_of

pytestmark = pytest.mark.gpu

FLOATS = ('ActionDensity', 'InternalEnergyDensity', 'WindingSquared')


def _check(got, c, s, where):
    for k in FLOATS:
        np.testing.assert_allclose(got[k], c[k][s], rtol=1e-12, err_msg=f'{where} {k} sweep {s}')
    assert (np.asarray(got['TorusWrapping']) == c['TorusWrapping'][s]).all(), f'{where} TorusWrapping sweep {s}'


@pytest.mark.parametrize('resident', [True, False])
@pytest.mark.parametrize('group', sorted(observable_groups()))
def test_single_lattice_inline_vs_reference(group, resident):
    for c in observable_groups()[group]:
        N = c['N']
        L = sv.Lattice2D(N)
        S = sv.Villain(L, c['kappa'], c['W'])
        G = sv.generator.villain.NeighborhoodUpdate(S, inline=True)
        G.rng = generator_from(c['rng0'])
        phi0, n0 = observable_start(c)
        start = {'phi': sv.Form(phi0[None].copy(), degree=0, lattice=L), 'n': sv.Form(n0.copy(), degree=1, lattice=L)}
        E = sv.Ensemble(S).generate(c['sweeps'], G, start=start, device_resident=resident)
        for s in range(c['sweeps']):
            got = {k: getattr(E.configuration, k).array[s] for k in FLOATS + ('TorusWrapping',)}
            _check(got, c, s, f'{group} seed {c["seed"]}')
        assert (state_of(G.rng) == c['rng1']).all()


@pytest.mark.parametrize('group', sorted(observable_groups()))
def test_replica_inline_vs_reference(group):
    chains = observable_groups()[group]
    R, N, kappa, W, sweeps = len(chains), chains[0]['N'], chains[0]['kappa'], chains[0]['W'], chains[0]['sweeps']
    starts = [observable_start(c) for c in chains]
    B = VillainReplicas(R, N, kappa, W)
    try:
        B.upload(np.stack([p for p, _ in starts]), np.stack([n for _, n in starts]))
        gens = [generator_from(c['rng0']) for c in chains]
        _, obs = B.run(sweeps, gens, inline=True)
    finally:
        B.close()
    for r, c in enumerate(chains):
        for s in range(sweeps):
            _check({k: obs[k][r, s] for k in obs}, c, s, f'{group} replica {r}')
        assert (state_of(gens[r]) == c['rng1']).all()
