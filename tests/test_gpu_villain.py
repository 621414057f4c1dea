"""NeighborhoodUpdate on the MI355X vs the reference's golden vectors and the CPU oracle.

Bar: phi and n bit-exact (np.array_equal), the NumPy bit-generator state after the call identical,
accepted counts exact, the float acceptance statistic within 1e-12 relative."""
import numpy as np
import pytest

import supervillain_amd as sv
from tests.golden import cases, crafted_generator, generator_from, state_of

pytestmark = pytest.mark.gpu


def run_gpu(N, kappa, W, phi0, n0, sweeps, gen, path=0, interval_phi=np.pi, interval_n=1, batched=False):
    L = sv.Lattice2D(N)
    S = sv.Villain(L, kappa, W)
    G = sv.generator.villain.NeighborhoodUpdate(S, interval_phi=interval_phi, interval_n=interval_n, path=path)
    G.rng = gen
    cfg = {'phi': sv.Form(phi0.reshape(1, N, N).copy(), degree=0, lattice=L),
           'n': sv.Form(n0.copy(), degree=1, lattice=L)}
    accepted, acceptance = [], []
    if batched:
        cfg = G._steps(cfg, sweeps)
    else:
        for _ in range(sweeps):
            cfg = G.step(cfg)
            accepted.append(G.accepted)
            acceptance.append(G.acceptance)
    return G, np.asarray(cfg['phi'])[0], np.asarray(cfg['n']), accepted, acceptance


@pytest.mark.parametrize('fixture', ['villain_neighborhood.npz', 'villain_rejections.npz'])
@pytest.mark.parametrize('path', [0, 1, 2])
def test_golden(fixture, path):
    for c in cases(fixture):
        if path == 2 and c['N'] % 2:
            continue
        G, phi, n, accepted, acceptance = run_gpu(c['N'], c['kappa'], c['W'], c['phi0'], c['n0'], c['sweeps'],
                                                  generator_from(c['rng0']), path, c['interval_phi'],
                                                  c['interval_n'])
        assert (phi == c['phi']).all(), (c['N'], c['kappa'], path)
        assert (n == c['n']).all()
        assert (state_of(G.rng) == c['rng1']).all()
        assert accepted == list(c['accepted'])
        np.testing.assert_allclose(acceptance, c['acceptance'], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize('path', [0, 2])
def test_golden_batched(path):
    """Many sweeps in one device call (the KeepEvery / bench path) equal the step-by-step chain."""
    for c in cases('villain_neighborhood.npz') + cases('villain_rejections.npz'):
        if c['N'] % 2:
            continue
        G, phi, n, _, _ = run_gpu(c['N'], c['kappa'], c['W'], c['phi0'], c['n0'], c['sweeps'],
                                  generator_from(c['rng0']), path, c['interval_phi'], c['interval_n'], batched=True)
        assert (phi == c['phi']).all() and (n == c['n']).all()
        assert (state_of(G.rng) == c['rng1']).all()
        assert G.accepted == c['accepted'][-1]


def hot(N, W, seed):
    r = np.random.default_rng(seed)
    return r.uniform(-np.pi, np.pi, (N, N)), W * r.integers(-2, 3, (2, N, N)).astype(np.int64)


@pytest.mark.parametrize('N', [4, 6, 10, 64, 126, 130, 250, 256])
@pytest.mark.parametrize('kappa', [0.1, 0.7])
def test_oracle_tiling(N, kappa, oracle_lib):
    """The fused kernel's strips/tiles (125-column strips, 64-row tiles, periodic halos) at sizes
    that do and do not divide evenly, against the oracle."""
    phi0, n0 = hot(N, 2, N)
    sweeps = 6
    G, phi, n, accepted, acceptance = run_gpu(N, kappa, 2, phi0, n0, sweeps, np.random.default_rng(N), path=2)
    g = np.random.default_rng(N)
    p, m = phi0.copy(), n0.copy()
    st = oracle_lib.villain_neighborhood(N, kappa, 2, p, m, sweeps, g)
    assert (phi == p).all() and (n == m).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert accepted[-1] == sum(s.accepted for s in st)


@pytest.mark.parametrize('N', [5, 7, 33, 101])
def test_oracle_odd(N, oracle_lib):
    phi0, n0 = hot(N, 1, N)
    G, phi, n, _, _ = run_gpu(N, 0.2, 1, phi0, n0, 4, np.random.default_rng(N))
    p, m = phi0.copy(), n0.copy()
    g = np.random.default_rng(N)
    oracle_lib.villain_neighborhood(N, 0.2, 1, p, m, 4, g)
    assert (phi == p).all() and (n == m).all() and G.rng.bit_generator.state == g.bit_generator.state


@pytest.mark.parametrize('path', [1, 2])
def test_forced_rejections_large(path, oracle_lib):
    """Forced Lemire rejections in several blocks of an N=128 sweep (including the last uint32 of a
    sweep, which carries the half-word buffer into the next sweep)."""
    N = 128
    V = N * N
    for pos, half in [(V + V // 2 + 7, 0), (V + V // 2 + V // 4 + 3, 1), (4 * V - 1, 1), (4 * V + V + V // 2 + 11, 0)]:
        phi0, n0 = hot(N, 1, pos)
        G, phi, n, _, _ = run_gpu(N, 0.3, 1, phi0, n0, 3, crafted_generator(pos % 1000, pos, half), path)
        g = crafted_generator(pos % 1000, pos, half)
        p, m = phi0.copy(), n0.copy()
        st = oracle_lib.villain_neighborhood(N, 0.3, 1, p, m, 3, g)
        assert sum(s.rejections for s in st) >= 1
        assert (phi == p).all() and (n == m).all() and G.rng.bit_generator.state == g.bit_generator.state


def test_fused_equals_generic_at_scale():
    """Two independent device implementations agree at N=1024 (size-independent property)."""
    N = 1024
    phi0, n0 = hot(N, 1, 11)
    _, p1, n1, a1, _ = run_gpu(N, 0.5, 1, phi0, n0, 3, np.random.default_rng(3), path=1)
    _, p2, n2, a2, _ = run_gpu(N, 0.5, 1, phi0, n0, 3, np.random.default_rng(3), path=2)
    assert (p1 == p2).all() and (n1 == n2).all() and a1 == a2


def test_constraint_and_counters_at_bench_size():
    """L=4096, W=2: the constraint dn = 0 mod W survives, counters are consistent."""
    N = 4096
    L = sv.Lattice2D(N)
    S = sv.Villain(L, 0.5, 2)
    G = sv.generator.villain.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(0)
    cfg = G._steps(S.configurations(1)[0], 4)
    assert G.sweeps == 4 and G.proposed == 4 * N * N and 0 < G.accepted < G.proposed
    assert S.valid(cfg)
    assert np.isfinite(S(cfg['phi'], cfg['n']))


def test_inline_observables_match_offline():
    N = 32
    L = sv.Lattice2D(N)
    S = sv.Villain(L, 0.4, 2)
    G = sv.generator.villain.NeighborhoodUpdate(S, inline=True)
    G.rng = np.random.default_rng(1)
    E = sv.Ensemble(S).generate(5, G)
    for i in range(5):
        phi, n = E.configuration[i]['phi'], E.configuration[i]['n']
        Sv = S(phi, n)
        np.testing.assert_allclose(E.configuration.ActionDensity.array[i], Sv / N ** 2, rtol=1e-12)
        np.testing.assert_allclose(E.configuration.InternalEnergyDensity.array[i], Sv / (N ** 2 * 0.4), rtol=1e-12)
        dn = sv.lattice.d(n)
        np.testing.assert_allclose(E.configuration.WindingSquared.array[i], np.mean(dn ** 2), rtol=1e-12)
        assert (E.configuration.TorusWrapping.array[i] == np.asarray(n).sum(axis=(1, 2))).all()


def test_ensemble_golden():
    c = [x for x in cases('ensemble.npz') if x['kind'] == 'villain_generate'][0]
    L = sv.Lattice2D(c['N'])
    S = sv.Villain(L, c['kappa'], c['W'])
    G = sv.generator.villain.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(c['seed'])
    E = sv.Ensemble(S).generate(c['steps'], G, starting_index=c['starting_index'], index_stride=c['index_stride'])
    assert (E.configuration.phi.array == c['phi']).all() and (E.configuration.n.array == c['n']).all()
    assert G.report() == c['report']
    c = [x for x in cases('ensemble.npz') if x['kind'] == 'keepevery_sequentially'][0]
    S = sv.Villain(L, c['kappa'], c['W'])
    a = sv.generator.villain.NeighborhoodUpdate(S)
    b = sv.generator.villain.NeighborhoodUpdate(S, interval_phi=1.0)
    a.rng, b.rng = np.random.default_rng(8), np.random.default_rng(9)
    G = sv.generator.KeepEvery(3, sv.generator.Sequentially((a, b)))
    E = sv.Ensemble(S).generate(c['steps'], G)
    assert (E.configuration.phi.array == c['phi']).all() and (E.configuration.n.array == c['n']).all()
    assert G.report() == c['report']


def test_config2_exact_parameters(oracle_lib):
    """BASELINE config 2 as stated: L=256, kappa=0.5, W=1 (interval_n=1), cold start, seed 0; 20 sweeps one per
    call (as Ensemble.generate makes them) against the oracle."""
    N, kappa, W, sweeps = 256, 0.5, 1, 20
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    G, phi, n, accepted, acceptance = run_gpu(N, kappa, W, phi0, n0, sweeps, np.random.default_rng(0), path=2)
    g = np.random.default_rng(0)
    p, m = phi0.copy(), n0.copy()
    st = oracle_lib.villain_neighborhood(N, kappa, W, p, m, sweeps, g)
    assert (phi == p).all() and (n == m).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert accepted[-1] == sum(s.accepted for s in st)
    np.testing.assert_allclose(acceptance[-1], sum(s.acceptance_sum for s in st) / N ** 2, rtol=1e-12)


def test_config2_batched_long_chain(oracle_lib):
    """Config 2's bench shape: 300 sweeps of L=256 (kappa=0.5, W=1) in one device call (several 64-sweep
    batches), against the oracle."""
    N, sweeps = 256, 300
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    G, phi, n, _, _ = run_gpu(N, 0.5, 1, phi0, n0, sweeps, np.random.default_rng(0), path=2, batched=True)
    g = np.random.default_rng(0)
    p, m = phi0.copy(), n0.copy()
    st = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, sweeps, g)
    assert (phi == p).all() and (n == m).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert G.accepted == sum(s.accepted for s in st)
