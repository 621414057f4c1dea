"""SiteUpdate, LinkUpdate, ExactUpdate, CohomologyUpdate on the MI355X vs the reference's
golden vectors (tests/golden/villain_generators.npz, incl. forced NumPy Lemire rejections) and, at sizes
whose grid-stride loops take several iterations per lane, vs the CPU oracle.

Bar: phi and n bit-exact, the NumPy bit-generator state after the call identical, accepted counts exact,
the float acceptance statistic within 1e-12 relative, report() text identical."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.generator import villain as gv
from tests.golden import cases, generator_from, state_of

pytestmark = pytest.mark.gpu

KINDS = {'SiteUpdate': gv.SiteUpdate, 'LinkUpdate': gv.LinkUpdate, 'ExactUpdate': gv.ExactUpdate,
         'CohomologyUpdate': gv.CohomologyUpdate}
KW = {'SiteUpdate': 'interval_phi', 'LinkUpdate': 'interval_n', 'ExactUpdate': 'interval_z',
      'CohomologyUpdate': 'interval_h'}


def make(kind, N, kappa, W, interval=None):
    S = sv.Villain(sv.Lattice2D(N), kappa, W)
    kw = {} if interval is None else {KW[kind]: interval}
    return S, KINDS[kind](S, **kw)


def golden_interval(c):
    if c['kw_interval'] == -1:
        return None
    return 0.7 if c['kind'] == 'SiteUpdate' else c['kw_interval']


def cfg_of(S, phi, n):
    N = S.Lattice.N
    return {'phi': sv.Form(phi.reshape(1, N, N).copy(), degree=0, lattice=S.Lattice),
            'n': sv.Form(n.reshape(2, N, N).copy(), degree=1, lattice=S.Lattice)}


@pytest.mark.parametrize('batched', [False, True])
def test_golden(batched):
    seen = set()
    for c in cases('villain_generators.npz'):
        N, kind = c['N'], c['kind']
        S, G = make(kind, N, c['kappa'], c['W'], golden_interval(c))
        G.rng = generator_from(c['rng0'])
        cfg = cfg_of(S, c['phi0'], c['n0'])
        accepted, acceptance = [], []
        if batched:
            cfg = G._steps(cfg, c['sweeps'])
        else:
            for _ in range(c['sweeps']):
                cfg = G.step(cfg)
                accepted.append(G.accepted)
                acceptance.append(G.acceptance)
        assert (np.asarray(cfg['phi']).reshape(N, N) == c['phi'].reshape(N, N)).all(), (kind, N)
        assert (np.asarray(cfg['n']).reshape(2, N, N) == c['n'].reshape(2, N, N)).all(), (kind, N)
        assert (state_of(G.rng) == c['rng1']).all(), (kind, N)
        if not batched:
            assert accepted == list(c['accepted']), (kind, N)
            np.testing.assert_allclose(acceptance, c['acceptance'], rtol=1e-12, atol=1e-15)
        assert G.accepted == c['accepted'][-1]
        np.testing.assert_allclose(G.acceptance, c['acceptance'][-1], rtol=1e-12, atol=1e-15)
        assert G.report() == c['report'], (kind, N)
        seen.add(kind)
    assert seen == set(KINDS)


def test_step_does_not_mutate_and_returns_only_its_fields():
    S, G = make('LinkUpdate', 8, 0.3, 1)
    G.rng = np.random.default_rng(3)
    phi0 = np.random.default_rng(4).uniform(-3, 3, (8, 8))
    cfg = cfg_of(S, phi0, np.zeros((2, 8, 8), dtype=np.int64)) | {'extra': 7}
    out = G.step(cfg)
    assert out['phi'] is cfg['phi'] and out['extra'] == 7
    assert (np.asarray(cfg['n']) == 0).all()
    assert np.asarray(out['n']).dtype == np.int64


@pytest.mark.parametrize('kind,N,sweeps,interval', [
    ('SiteUpdate', 2048, 2, None), ('SiteUpdate', 1030, 2, 1.3), ('SiteUpdate', 33, 3, None),
    ('ExactUpdate', 2048, 2, None), ('ExactUpdate', 1030, 2, 3), ('ExactUpdate', 33, 3, 2),
    ('LinkUpdate', 1024, 2, None), ('LinkUpdate', 700, 2, 3), ('LinkUpdate', 33, 3, 2),
    ('CohomologyUpdate', 4096, 4, None), ('CohomologyUpdate', 1000, 4, 3), ('CohomologyUpdate', 129, 8, 1),
])
def test_large_vs_oracle(oracle_lib, kind, N, sweeps, interval):
    """Lattices big enough that each lane loops (stride maps), odd N, non-power-of-two N."""
    kappa, W = 0.45, 1
    S, G = make(kind, N, kappa, W, interval)
    rs = np.random.default_rng(N)
    phi = rs.uniform(-np.pi, np.pi, (N, N))
    n = rs.integers(-2, 3, (2, N, N)).astype(np.int64)
    G.rng = np.random.default_rng(11 + N)
    cfg = G._steps(cfg_of(S, phi, n), sweeps)
    g = np.random.default_rng(11 + N)
    po, no = phi.copy(), n.copy()
    st = oracle_lib.villain_generator(kind, N, kappa, W, po, no, sweeps, g, interval)
    assert (np.asarray(cfg['phi']).reshape(N, N) == po).all()
    assert (np.asarray(cfg['n']).reshape(2, N, N) == no).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert G.accepted == sum(s.accepted for s in st)


def test_hammer_sequence_vs_oracle(oracle_lib):
    """The Hammer, Sequentially(Site, Link, Exact, Cohomology, Worm), over several steps."""
    N, kappa, W = 64, 0.6, 2
    S = sv.Villain(sv.Lattice2D(N), kappa, W)
    H = gv.Hammer(S)
    seeds = [21, 22, 23, 24, 25]
    for G, s in zip(H.generators, seeds):
        G.rng = np.random.default_rng(s)
    cfg = cfg_of(S, np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64))
    for _ in range(3):
        cfg = H.step(cfg)
    gens = [np.random.default_rng(s) for s in seeds]
    phi, n = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    for _ in range(3):
        for kind, g in zip(['SiteUpdate', 'LinkUpdate', 'ExactUpdate', 'CohomologyUpdate'], gens):
            oracle_lib.villain_generator(kind, N, kappa, W, phi, n, 1, g)
        hist, lengths = oracle_lib.villain_worm(N, kappa, W, phi, n, 1, gens[4])
    assert (np.asarray(cfg['Vortex_Vortex']) == hist).all() and cfg['Worm_Length'] == lengths[-1]
    assert (np.asarray(cfg['phi']).reshape(N, N) == phi).all()
    assert (np.asarray(cfg['n']) == n).all()
