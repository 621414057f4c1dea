"""VortexUpdate and WrappingUpdate on the MI355X vs the reference's golden vectors
(tests/golden/worldline_generators.npz: finite and infinite W, forced NumPy Lemire rejections) and, at sizes
whose grid-stride loops and LDS-staged column sums take several iterations, vs the CPU oracle.

Bar: m and v bit-exact (float v at W = infinity included), the NumPy bit-generator state identical, accepted
counts exact, the float acceptance statistic within 1e-12 relative, report() text identical."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.generator import worldline as gw
from tests.golden import cases, generator_from, state_of

pytestmark = pytest.mark.gpu

KINDS = {'VortexUpdate': (gw.VortexUpdate, 'interval_v'), 'WrappingUpdate': (gw.WrappingUpdate, 'interval_w')}


def make(kind, N, kappa, W, interval=None):
    S = sv.Worldline(sv.Lattice2D(N), kappa, W)
    cls, kw = KINDS[kind]
    return S, cls(S, **({} if interval is None else {kw: interval}))


def cfg_of(S, m, v):
    N = S.Lattice.N
    return {'m': sv.Form(m.reshape(2, N, N).copy(), degree=1, lattice=S.Lattice),
            'v': sv.Form(v.reshape(1, N, N).copy(), degree=2, lattice=S.Lattice)}


@pytest.mark.parametrize('batched', [False, True])
def test_golden(batched):
    seen = set()
    for c in cases('worldline_generators.npz'):
        N, kind = c['N'], c['kind']
        S, G = make(kind, N, c['kappa'], c['W'], None if c['kw_interval'] == -1 else c['kw_interval'])
        G.rng = generator_from(c['rng0'])
        cfg = cfg_of(S, c['m0'], c['v0'])
        accepted, acceptance = [], []
        if batched:
            cfg = cfg | G._steps(cfg, c['sweeps'])
        else:
            for _ in range(c['sweeps']):
                cfg = cfg | G.step(cfg)
                accepted.append(G.accepted)
                acceptance.append(G.acceptance)
        assert (np.asarray(cfg['m']) == c['m']).all(), (kind, N, c['W'])
        assert (np.asarray(cfg['v']).reshape(N, N) == c['v']).all(), (kind, N, c['W'])
        assert (state_of(G.rng) == c['rng1']).all(), (kind, N)
        if not batched:
            assert accepted == list(c['accepted']), (kind, N)
            np.testing.assert_allclose(acceptance, c['acceptance'], rtol=1e-12, atol=1e-15)
        assert G.accepted == c['accepted'][-1]
        assert G.report() == c['report'], (kind, N)
        seen.add(kind)
    assert seen == set(KINDS)


@pytest.mark.parametrize('kind,N,W,sweeps,interval', [
    ('VortexUpdate', 2048, 1, 2, None), ('VortexUpdate', 1030, 2, 2, 3), ('VortexUpdate', 33, 1, 3, 2),
    ('VortexUpdate', 1024, float('inf'), 2, None), ('VortexUpdate', 31, float('inf'), 3, 2),
    ('WrappingUpdate', 4096, 1, 3, None), ('WrappingUpdate', 1000, 3, 3, 2), ('WrappingUpdate', 129, 1, 4, 3),
    ('WrappingUpdate', 777, float('inf'), 3, None), ('WrappingUpdate', 7, 2, 5, 1),
])
def test_large_vs_oracle(oracle_lib, kind, N, W, sweeps, interval):
    kappa = 0.35
    S, G = make(kind, N, kappa, W, interval)
    rs = np.random.default_rng(N + 5)
    m = rs.integers(-2, 3, (2, N, N)).astype(np.int64)
    v = rs.standard_normal((N, N)) if not np.isfinite(W) else (W * rs.integers(-2, 3, (N, N))).astype(np.int64)
    G.rng = np.random.default_rng(70 + N)
    cfg = cfg_of(S, m, v)
    cfg = cfg | G._steps(cfg, sweeps)
    g = np.random.default_rng(70 + N)
    mo, vo = m.copy(), v.copy()
    st = oracle_lib.worldline_generator(kind, N, kappa, S._W, mo, vo, sweeps, g, interval)
    assert (np.asarray(cfg['m']) == mo).all()
    assert (np.asarray(cfg['v']).reshape(N, N) == vo).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert G.accepted == sum(s.accepted for s in st)


def test_hammer_sequence():
    """The Worldline Hammer: Sequentially(Vortex, Coexact, Wrapping, Worm) vs the four generators
    stepped by hand with the same streams."""
    N, kappa, W = 32, 0.5, 1
    S = sv.Worldline(sv.Lattice2D(N), kappa, W)
    H = gw.Hammer(S)
    seeds = [31, 32, 33, 34]
    for G, s in zip(H.generators, seeds):
        G.rng = np.random.default_rng(s)
    cfg = cfg_of(S, np.zeros((2, N, N), dtype=np.int64), np.zeros((N, N), dtype=np.int64))
    for _ in range(3):
        cfg = H.step(cfg)
    gens = [gw.VortexUpdate(S), gw.CoexactUpdate(S), gw.WrappingUpdate(S), gw.ClassicWorm(S)]
    for G, s in zip(gens, seeds):
        G.rng = np.random.default_rng(s)
    c2 = cfg_of(S, np.zeros((2, N, N), dtype=np.int64), np.zeros((N, N), dtype=np.int64))
    for _ in range(3):
        for G in gens:
            c2 = c2 | G.step(c2)
    assert (np.asarray(cfg['m']) == np.asarray(c2['m'])).all()
    assert (np.asarray(cfg['v']) == np.asarray(c2['v'])).all()
    assert (np.asarray(cfg['Spin_Spin']) == np.asarray(c2['Spin_Spin'])).all()
    assert gens[3].report() == H.generators[3].report()
    assert H.generators[0].accepted + H.generators[2].accepted > 0
