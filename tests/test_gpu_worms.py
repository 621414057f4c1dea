"""both ClassicWorms on the GPU (supervillain_amd/csrc/worm.hip) against the reference's
golden steps (tests/golden/worms.npz) and the oracle (batches of replicas, one chain per lane)."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.generator import villain as gv, worldline as gw
from supervillain_amd.replicas import VillainReplicas, worldline_worms
from tests.golden import cases, generator_from, state_of

pytestmark = pytest.mark.gpu


def test_worms_golden():
    """The generators, step by step, against the reference: every histogram, length, final field, rng, report."""
    for c in cases('worms.npz'):
        if c['action'].startswith('hammer'):
            continue
        N = c['N']
        L = sv.Lattice2D(N)
        if c['action'] == 'villain':
            S = sv.Villain(L, c['kappa'], c['W'])
            G = gv.Worm(S)
            cfg = {'phi': sv.Form(c['phi0'][None], degree=0, lattice=L), 'n': sv.Form(c['n0'], degree=1, lattice=L)}
            key, field = 'Vortex_Vortex', 'n'
        else:
            S = sv.Worldline(L, c['kappa'], c['W'])
            G = gw.Worm(S)
            cfg = {'m': sv.Form(c['m0'], degree=1, lattice=L), 'v': sv.Form(c['v0'][None], degree=2, lattice=L)}
            key, field = 'Spin_Spin', 'm'
        assert str(G) == 'ClassicWorm'
        G.rng = generator_from(c['rng0'])
        for k in range(c['steps']):
            cfg = G.step(cfg)
            assert (np.asarray(cfg[key]) == c['hist'][k]).all(), (c['action'], N, k)
            assert cfg['Worm_Length'] == c['lengths'][k]
        assert (np.asarray(cfg[field]) == c[field]).all()
        assert (state_of(G.rng) == c['rng1']).all()
        assert G.report() == c['report']


def thermalized_villain(oracle_lib, R, N, kappa, W, seed):
    phi = np.zeros((R, N, N))
    n = np.zeros((R, 2, N, N), dtype=np.int64)
    for r in range(R):
        oracle_lib.villain_neighborhood(N, kappa, W, phi[r], n[r], 10, np.random.default_rng(seed + r))
    return phi, n


@pytest.mark.parametrize('R,N,kappa,W', [(130, 16, 0.5, 1), (70, 12, 0.7, 2), (64, 8, 1.1, 3)])
def test_villain_replica_worms(oracle_lib, R, N, kappa, W):
    """R chains (not a multiple of the 64-lane wave), 3 worms each, every chain == the oracle with its own stream."""
    phi, n = thermalized_villain(oracle_lib, R, N, kappa, W, 100)
    B = VillainReplicas(R, N, kappa, W)
    B.upload(phi, n)
    rngs = [np.random.default_rng(1000 + r) for r in range(R)]
    hist, lengths = B.worm(rngs, worms=3)
    phi1, n1 = B.download()
    assert (phi1 == phi).all()
    for r in range(R):
        g = np.random.default_rng(1000 + r)
        nr = n[r].copy()
        h, l = oracle_lib.villain_worm(N, kappa, W, phi[r], nr, 3, g)
        assert (nr == n1[r]).all() and (h == hist[r]).all() and (l == lengths[r]).all(), r
        assert g.bit_generator.state == rngs[r].bit_generator.state
    B.close()


@pytest.mark.parametrize('W', [1, 2, float('inf')])
def test_worldline_replica_worms(oracle_lib, W):
    R, N, kappa = 96, 10, 0.6
    m = np.zeros((R, 2, N, N), dtype=np.int64)
    r0 = np.random.default_rng(5)
    W_eff = 2 * np.pi if W == float('inf') else float(W)
    v = r0.standard_normal((R, N, N)) if W == float('inf') else (int(W) * r0.integers(-2, 3, (R, N, N))).astype(np.int64)
    for r in range(R):
        oracle_lib.worldline_coexact(N, kappa, W_eff, m[r], v[r], 10, np.random.default_rng(300 + r))
    m0 = m.copy()
    rngs = [np.random.default_rng(2000 + r) for r in range(R)]
    hist, lengths = worldline_worms(m, v, kappa, W, rngs, worms=2)
    for r in range(R):
        g = np.random.default_rng(2000 + r)
        mr = m0[r].copy()
        h, l = oracle_lib.worldline_worm(N, kappa, W_eff, mr, v[r], 2, g)
        assert (mr == m[r]).all() and (h == hist[r]).all() and (l == lengths[r]).all(), r
        assert g.bit_generator.state == rngs[r].bit_generator.state


def test_worm_max_moves_is_an_error():
    S = sv.Worldline(sv.Lattice2D(8), 2.0, 1)
    G = gw.Worm(S, max_moves=1)
    G.rng = np.random.default_rng(0)
    cfg = {'m': sv.Form(np.zeros((2, 8, 8), dtype=np.int64), degree=1, lattice=S.Lattice),
           'v': sv.Form(np.zeros((1, 8, 8), dtype=np.int64), degree=2, lattice=S.Lattice)}
    with pytest.raises(Exception, match='max_moves'):
        for _ in range(50):
            cfg = G.step(cfg)



def test_hammer_ensemble_golden():
    """Ensemble(S).generate(steps, Hammer(S, worms)) -- every member generator of the reference's Hammer, the
    worm included (KeepEvery-blocked histogram average for worms > 1) -- against the reference's own run."""
    from supervillain_amd.generator.combining import KeepEvery
    for c in cases('worms.npz'):
        if not c['action'].startswith('hammer'):
            continue
        villain = c['action'] == 'hammer_villain'
        L = sv.Lattice2D(c['N'])
        S = (sv.Villain if villain else sv.Worldline)(L, c['kappa'], c['W'])
        H = (gv if villain else gw).Hammer(S, c['worms'])
        for G, seed in zip(H.generators, c['seeds']):
            (G.generator if isinstance(G, KeepEvery) else G).rng = np.random.default_rng(int(seed))
        E = sv.Ensemble(S).generate(c['steps'], H)
        arr = lambda x: np.asarray(x.array if hasattr(x, 'array') else x)
        for f in (('phi', 'n') if villain else ('m', 'v')):
            assert (arr(getattr(E, f)) == c[f]).all(), (c['action'], f)
        assert (arr(getattr(E, 'Vortex_Vortex' if villain else 'Spin_Spin')) == c['hist']).all(), c['action']
        assert (arr(E.Worm_Length) == c['lengths']).all(), c['action']
        assert H.report() == c['report']


@pytest.mark.parametrize('N', [2, 3])
def test_tiny_lattices(oracle_lib, N):
    """N = 2, 3 (every neighbour wraps; FFT coordinates fold onto themselves) for both worms, W = 1 and 2.
    (Replica batches of the Villain sweep need an even N >= 4, so the Villain worm runs as the generator.)"""
    for W in (1, 2):
        L = sv.Lattice2D(N)
        S = sv.Villain(L, 0.8, W)
        for r in range(3):
            phi = np.random.default_rng(N + r).uniform(-np.pi, np.pi, (1, N, N))
            G = gv.Worm(S)
            G.rng = np.random.default_rng(50 + r)
            cfg = {'phi': sv.Form(phi, degree=0, lattice=L), 'n': sv.Form(np.zeros((2, N, N), dtype=np.int64), degree=1,
                                                                          lattice=L)}
            g = np.random.default_rng(50 + r)
            n = np.zeros((2, N, N), dtype=np.int64)
            for _ in range(6):
                cfg = G.step(cfg)
                h, l = oracle_lib.villain_worm(N, 0.8, W, phi[0], n, 1, g)
                assert (np.asarray(cfg['n']) == n).all() and (np.asarray(cfg['Vortex_Vortex']) == h).all()
                assert cfg['Worm_Length'] == l[0]
        R = 5
        m = np.zeros((R, 2, N, N), dtype=np.int64)
        v = (W * np.random.default_rng(N + 1).integers(-1, 2, (R, N, N))).astype(np.int64)
        rngs = [np.random.default_rng(70 + r) for r in range(R)]
        hist, lengths = worldline_worms(m, v, 0.8, W, rngs, worms=6)
        for r in range(R):
            mr = np.zeros((2, N, N), dtype=np.int64)
            h, l = oracle_lib.worldline_worm(N, 0.8, float(W), mr, v[r], 6, np.random.default_rng(70 + r))
            assert (mr == m[r]).all() and (h == hist[r]).all() and (l == lengths[r]).all()
