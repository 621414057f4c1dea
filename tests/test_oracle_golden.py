"""Pin the CPU oracle (oracle/sv_oracle.c) to golden vectors captured from the reference.

The oracle is only trusted as the GPU path's checker because of these tests.
"""
import numpy as np
import pytest

from tests.golden import cases, generator_from, state_of


def test_rng_kat(oracle_lib):
    O = oracle_lib
    for c in cases('rng_kat.npz'):
        g = generator_from(c['rng0'])
        if len(c['raw']):
            assert (O.raw(g, len(c['raw'])) == c['raw']).all()
        assert (O.uniform(g, 0.0, 1.0, len(c['uniform01'])) == c['uniform01']).all()
        if len(c['uniform_pi']):
            assert (O.uniform(g, -np.pi, np.pi, len(c['uniform_pi'])) == c['uniform_pi']).all()
        assert (O.integers(g, 3, len(c['choice3'])) - 1 == c['choice3']).all()
        assert (O.uniform(g, 0.0, 1.0, len(c['uniform_after'])) == c['uniform_after']).all()
        assert (2 * O.integers(g, 2, len(c['choice2'])) - 1 == c['choice2']).all()
        assert (O.integers(g, 5, len(c['choice5'])) - 2 == c['choice5']).all()
        assert (state_of(g) == c['rng1']).all()


def test_checkerboarding(oracle_lib):
    for c in cases('checkerboarding.npz'):
        ncol, col = oracle_lib.colors(c['N'])
        assert ncol == c['colors'].max() + 1
        assert (col == c['colors']).all()


def _villain(O, c):
    g = generator_from(c['rng0'])
    phi, n = c['phi0'].copy(), c['n0'].copy()
    st = O.villain_neighborhood(c['N'], c['kappa'], c['W'], phi, n, c['sweeps'], g,
                                interval_phi=c['interval_phi'], interval_n=c['interval_n'])
    return g, phi, n, st


@pytest.mark.parametrize('fixture', ['villain_neighborhood.npz', 'villain_rejections.npz'])
def test_villain_neighborhood(oracle_lib, fixture):
    for c in cases(fixture):
        g, phi, n, st = _villain(oracle_lib, c)
        assert (phi == c['phi']).all(), (c['N'], c['kappa'])
        assert (n == c['n']).all()
        assert (state_of(g) == c['rng1']).all()
        assert np.cumsum([s.accepted for s in st])[-1] == c['accepted'][-1]
        V = c['N'] ** 2
        acc = np.cumsum([s.acceptance_sum / V for s in st])
        np.testing.assert_allclose(acc, c['acceptance'], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(oracle_lib.villain_action(c['N'], c['kappa'], phi, n), c['action'], rtol=1e-12)


def test_rejection_fixtures_really_reject(oracle_lib):
    hit = 0
    for c in cases('villain_rejections.npz'):
        _, _, _, st = _villain(oracle_lib, c)
        hit += sum(s.rejections for s in st) > 0
    assert hit >= 6


def test_worldline_coexact(oracle_lib):
    for c in cases('worldline_coexact.npz'):
        g = generator_from(c['rng0'])
        m = np.zeros((2, c['N'], c['N']), dtype=np.int64)
        st = oracle_lib.worldline_coexact(c['N'], c['kappa'], c['W_eff'], m, np.ascontiguousarray(c['v']),
                                          c['sweeps'], g, interval_t=c['interval_t'])
        assert (m == c['m']).all(), (c['N'], c['W'])
        assert (state_of(g) == c['rng1']).all()
        assert np.cumsum([s.accepted for s in st])[-1] == c['accepted'][-1]
        V = c['N'] ** 2
        np.testing.assert_allclose(np.cumsum([s.acceptance_sum / V for s in st]), c['acceptance'], rtol=1e-12)


def test_worldline_plaquette_sequential(oracle_lib):
    for c in cases('worldline_plaquette.npz'):
        N = c['N']
        g = generator_from(c['rng0'])
        m = np.zeros((2, N, N), dtype=np.int64)
        v = np.zeros((N, N), dtype=np.float64 if np.isinf(c['W']) else np.int64)
        acc, tot = 0, 0.0
        for k in range(c['sweeps']):
            st = oracle_lib.worldline_plaquette_seq(N, c['kappa'], c['W_eff'], m, v, c['order'][k], g)
            acc += st.accepted
            tot += st.acceptance_sum
            assert acc == c['accepted'][k]
            np.testing.assert_allclose(tot, c['acceptance'][k], rtol=1e-12)
        assert (m == c['m']).all() and (v == c['v']).all()
        assert (state_of(g) == c['rng1']).all()


ACCEPTANCE_DENOMINATOR = {'SiteUpdate': lambda N: N * N, 'ExactUpdate': lambda N: N * N,
                          'LinkUpdate': lambda N: 2 * N * N, 'CohomologyUpdate': lambda N: 2}


def generator_interval(c):
    if c['kw_interval'] == -1:
        return None
    return 0.7 if c['kind'] == 'SiteUpdate' else c['kw_interval']


def test_villain_generators_golden(oracle_lib):
    """SiteUpdate, LinkUpdate, ExactUpdate, CohomologyUpdate chains from the reference
    (including forced NumPy Lemire rejections) reproduced bit-for-bit by the oracle."""
    kinds = set()
    for c in cases('villain_generators.npz'):
        N, kind = c['N'], c['kind']
        phi, n = c['phi0'].reshape(N, N).copy(), c['n0'].reshape(2, N, N).copy()
        g = generator_from(c['rng0'])
        st = oracle_lib.villain_generator(kind, N, c['kappa'], c['W'], phi, n, c['sweeps'], g, generator_interval(c))
        assert (phi == c['phi'].reshape(N, N)).all() and (n == c['n'].reshape(2, N, N)).all(), (kind, N)
        assert (state_of(g) == c['rng1']).all()
        assert list(np.cumsum([s.accepted for s in st])) == list(c['accepted'])
        d = ACCEPTANCE_DENOMINATOR[kind](N)
        np.testing.assert_allclose(np.cumsum([s.acceptance_sum / d for s in st]), c['acceptance'], rtol=1e-12)
        kinds.add(kind)
    assert kinds == set(ACCEPTANCE_DENOMINATOR)


WORLDLINE_DENOMINATOR = {'VortexUpdate': lambda N: N * N, 'WrappingUpdate': lambda N: 2 * N}


def test_worldline_generators_golden(oracle_lib):
    """VortexUpdate and WrappingUpdate chains from the reference (finite and infinite W,
    forced NumPy Lemire rejections) reproduced bit-for-bit by the oracle."""
    kinds = set()
    for c in cases('worldline_generators.npz'):
        N, kind = c['N'], c['kind']
        m, v = c['m0'].copy(), np.ascontiguousarray(c['v0'])
        g = generator_from(c['rng0'])
        iv = None if c['kw_interval'] == -1 else c['kw_interval']
        st = oracle_lib.worldline_generator(kind, N, c['kappa'], c['W_eff'], m, v, c['sweeps'], g, iv)
        assert (m == c['m']).all() and (v == c['v']).all(), (kind, N, c['W'])
        assert (state_of(g) == c['rng1']).all(), (kind, N)
        assert list(np.cumsum([s.accepted for s in st])) == list(c['accepted']), (kind, N)
        d = WORLDLINE_DENOMINATOR[kind](N)
        np.testing.assert_allclose(np.cumsum([s.acceptance_sum / d for s in st]), c['acceptance'], rtol=1e-12)
        kinds.add(kind)
    assert kinds == set(WORLDLINE_DENOMINATOR)
    assert sum(1 for c in cases('worldline_generators.npz') if c['kw_interval'] == 3) >= 4  # rejection cases


def test_worms_golden(oracle_lib):
    """both ClassicWorms, step by step (every step's histogram and length)."""
    O = oracle_lib
    for c in cases('worms.npz'):
        if c['action'].startswith('hammer'):
            continue  # whole-Hammer Ensemble fixtures: tests/test_gpu_worms.py
        N, g = c['N'], generator_from(c['rng0'])
        for k in range(c['steps']):
            if c['action'] == 'villain':
                n = c['n0'].copy() if k == 0 else n
                hist, lengths = O.villain_worm(N, c['kappa'], c['W'], c['phi0'], n, 1, g)
            else:
                m = c['m0'].copy() if k == 0 else m
                hist, lengths = O.worldline_worm(N, c['kappa'], c['W_eff'], m, np.ascontiguousarray(c['v0']), 1, g)
            assert (hist == c['hist'][k]).all(), (c['action'], N, k)
            assert lengths[0] == c['lengths'][k] == hist.sum()
        assert ((n if c['action'] == 'villain' else m) == (c['n'] if c['action'] == 'villain' else c['m'])).all()
        assert (state_of(g) == c['rng1']).all()


def test_multicore_oracle_matches(oracle_lib):
    """The OpenMP restatement (bench.py's multi-core CPU baseline) is the same chain: the reference's golden
    rejection fixtures (forced NumPy Lemire rejections -> the sequential fallback) and plain seeded chains."""
    O = oracle_lib
    checked = 0
    for c in cases('villain_rejections.npz'):
        if c['N'] % 2:
            continue
        checked += 1
        phi, n = c['phi0'].copy(), c['n0'].copy()
        g = generator_from(c['rng0'])
        O.villain_neighborhood_mt(c['N'], c['kappa'], c['W'], phi, n, c['sweeps'], g, 4,
                                  interval_phi=c['interval_phi'], interval_n=c['interval_n'])
        assert (phi == c['phi']).all() and (n == c['n']).all() and (state_of(g) == c['rng1']).all()
    assert checked >= 4
    for N, W in [(32, 1), (20, 2)]:
        a = [np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64), np.random.default_rng(N)]
        b = [np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64), np.random.default_rng(N)]
        O.villain_neighborhood(N, 0.4, W, a[0], a[1], 5, a[2])
        O.villain_neighborhood_mt(N, 0.4, W, b[0], b[1], 5, b[2], 3)
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
        assert a[2].bit_generator.state == b[2].bit_generator.state


def _offline_observables(phi, n, kappa):
    """(ActionDensity, InternalEnergyDensity, WindingSquared, TorusWrapping) of one Villain configuration, restated
    from observable/action.py:25-31, energy.py:25-30, winding.py:30-37, wrapping.py:17-25 and action/villain.py:51-66."""
    N = phi.shape[0]
    l0 = (0.0 + (np.roll(phi, -1, axis=0) - phi)) - 2 * np.pi * n[0]
    l1 = (0.0 + (np.roll(phi, -1, axis=1) - phi)) - 2 * np.pi * n[1]
    S = kappa / 2 * ((l0 ** 2).sum() + (l1 ** 2).sum())
    dn = (np.roll(n[1], -1, axis=0) - n[1]) - (np.roll(n[0], -1, axis=1) - n[0])
    return S / N ** 2, S / (N ** 2 * kappa), (dn ** 2).mean(), n.sum(axis=(1, 2))


def test_observables_golden(oracle_lib):
    """The oracle's chain, measured after every sweep, gives the reference's own observable values
    (tests/golden/villain_observables.npz, tools/make_golden_observables.py): the fixture the GPU's inline
    observables are compared with is the oracle's chain."""
    from tests.golden import observable_start
    for c in cases('villain_observables.npz'):
        g = generator_from(c['rng0'])
        phi, n = observable_start(c)
        for s in range(c['sweeps']):
            oracle_lib.villain_neighborhood(c['N'], c['kappa'], c['W'], phi, n, 1, g)
            ad, ie, w2, tw = _offline_observables(phi, n, c['kappa'])
            np.testing.assert_allclose(ad, c['ActionDensity'][s], rtol=1e-12)
            np.testing.assert_allclose(ie, c['InternalEnergyDensity'][s], rtol=1e-12)
            np.testing.assert_allclose(w2, c['WindingSquared'][s], rtol=1e-12)
            assert (tw == c['TorusWrapping'][s]).all()
        assert (state_of(g) == c['rng1']).all()
