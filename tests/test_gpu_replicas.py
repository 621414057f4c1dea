"""Replica batches (sv_replicas_*, BASELINE config 5) on the MI355X: every replica is bit-for-bit the
single chain its generator gives (CPU oracle), Lemire rejections in one replica leave the others
alone, and the inline observables equal the offline measurement of each configuration (integers
exactly, the action within 1e-12 relative)."""
import numpy as np
import pytest

from supervillain_amd.replicas import VillainReplicas
from tests.golden import crafted_generator

pytestmark = pytest.mark.gpu


def hot(R, N, W, seed):
    r = np.random.default_rng(seed)
    return r.uniform(-np.pi, np.pi, (R, N, N)), W * r.integers(-2, 3, (R, 2, N, N)).astype(np.int64)


def offline(phi, n):
    """(sum (d phi - 2 pi n)^2, sum (dn)^2, sum n0, sum n1) of one configuration (villain.py:51-66,
    winding.py:30-37, wrapping.py:17-25)."""
    l0 = (0.0 + (np.roll(phi, -1, axis=0) - phi)) - 2 * np.pi * n[0]
    l1 = (0.0 + (np.roll(phi, -1, axis=1) - phi)) - 2 * np.pi * n[1]
    dn = (np.roll(n[1], -1, axis=0) - n[1]) - (np.roll(n[0], -1, axis=1) - n[0])
    return (l0 ** 2).sum() + (l1 ** 2).sum(), (dn ** 2).sum(), n[0].sum(), n[1].sum()


def run_batch(R, N, kappa, W, phi0, n0, sweeps, gens, inline=False):
    B = VillainReplicas(R, N, kappa, W)
    try:
        B.upload(phi0, n0)
        stats, obs = B.run(sweeps, gens, inline=inline)
        phi, n = B.download()
    finally:
        B.close()
    return phi, n, stats, obs


@pytest.mark.parametrize('N,sweeps', [(16, 5), (64, 70), (128, 3), (130, 2), (256, 2)])
def test_each_replica_is_its_own_chain(N, sweeps, oracle_lib):
    R = 5
    phi0, n0 = hot(R, N, 2, N)
    gens = [np.random.default_rng(100 + r) for r in range(R)]
    phi, n, stats, _ = run_batch(R, N, 0.5, 2, phi0, n0, sweeps, gens)
    for r in range(R):
        g = np.random.default_rng(100 + r)
        p, m = phi0[r].copy(), n0[r].copy()
        st = oracle_lib.villain_neighborhood(N, 0.5, 2, p, m, sweeps, g)
        assert (phi[r] == p).all() and (n[r] == m).all(), r
        assert gens[r].bit_generator.state == g.bit_generator.state
        assert list(stats['accepted'][r]) == [s.accepted for s in st]
        np.testing.assert_allclose(stats['acceptance'][r], [s.acceptance_sum / N ** 2 for s in st], rtol=1e-12)


def test_rejection_in_one_replica(oracle_lib):
    """Replica 2 meets forced Lemire rejections (one in a choice block, one at a sweep's last uint32);
    every replica still equals its own chain."""
    R, N = 4, 32
    V = N * N
    phi0, n0 = hot(R, N, 1, 9)
    for pos, half in [(V + V // 2 + 9, 0), (4 * V - 1, 1), (4 * V + V + V // 2 + 3, 1)]:
        def gens_():
            return [crafted_generator(7, pos, half) if r == 2 else np.random.default_rng(r) for r in range(R)]
        gens = gens_()
        phi, n, stats, _ = run_batch(R, N, 0.4, 1, phi0, n0, 3, gens)
        ref = gens_()
        for r in range(R):
            p, m = phi0[r].copy(), n0[r].copy()
            st = oracle_lib.villain_neighborhood(N, 0.4, 1, p, m, 3, ref[r])
            assert (phi[r] == p).all() and (n[r] == m).all(), (pos, r)
            assert gens[r].bit_generator.state == ref[r].bit_generator.state
            assert list(stats['rejections'][r]) == [s.rejections for s in st]
        assert stats['rejections'][2].sum() >= 1


@pytest.mark.parametrize('inline', [False, True])
def test_rejections_in_later_batches(oracle_lib, inline):
    """Several 64-sweep batches (two in flight: the next one is enqueued before the current one has finished):
    forced Lemire rejections in the second batch's 7th sweep, the first sweep of the third batch and the last
    sweep of the call; every replica equals its own chain, with its statistics and inline observables."""
    R, N, sweeps, kappa = 4, 16, 150, 0.4
    V = N * N
    phi0, n0 = hot(R, N, 1, 21)
    crafted = {1: (70 * 4 * V + V + V // 2 + 9, 0), 2: (128 * 4 * V + 3 * V + 7, 1), 3: (149 * 4 * V + 3 * V + 1, 0)}

    def gens_():
        return [crafted_generator(30 + r, *crafted[r]) if r in crafted else np.random.default_rng(r) for r in range(R)]
    gens = gens_()
    phi, n, stats, obs = run_batch(R, N, kappa, 1, phi0, n0, sweeps, gens, inline=inline)
    ref = gens_()
    for r in range(R):
        p, m = phi0[r].copy(), n0[r].copy()
        st = oracle_lib.villain_neighborhood(N, kappa, 1, p, m, sweeps, ref[r])
        assert (phi[r] == p).all() and (n[r] == m).all(), r
        assert gens[r].bit_generator.state == ref[r].bit_generator.state
        assert list(stats['accepted'][r]) == [s.accepted for s in st]
        assert list(stats['rejections'][r]) == [s.rejections for s in st]
        if inline:
            act, w2, s0, s1 = offline(p, m)
            np.testing.assert_allclose(obs['ActionDensity'][r, -1], kappa / 2 * act / V, rtol=1e-12)
            assert obs['WindingSquared'][r, -1] == w2 / V
            assert list(obs['TorusWrapping'][r, -1]) == [s0, s1]
    for r in crafted:
        assert stats['rejections'][r].sum() >= 1, r


def test_inline_observables_match_offline(oracle_lib):
    R, N, sweeps, kappa = 3, 32, 4, 0.5
    phi0, n0 = hot(R, N, 2, 4)
    gens = [np.random.default_rng(r) for r in range(R)]
    _, _, _, obs = run_batch(R, N, kappa, 2, phi0, n0, sweeps, gens, inline=True)
    V = N * N
    for r in range(R):
        g = np.random.default_rng(r)
        p, m = phi0[r].copy(), n0[r].copy()
        for k in range(sweeps):
            oracle_lib.villain_neighborhood(N, kappa, 2, p, m, 1, g)
            act, w2, s0, s1 = offline(p, m)
            np.testing.assert_allclose(obs['ActionDensity'][r, k], kappa / 2 * act / V, rtol=1e-12)
            np.testing.assert_allclose(obs['InternalEnergyDensity'][r, k], act / 2 / V, rtol=1e-12)
            assert obs['WindingSquared'][r, k] == w2 / V
            assert list(obs['TorusWrapping'][r, k]) == [s0, s1]


def test_config5_shape_against_single_chains():
    """128 replicas of L=128 at W=2 (one GPU's share of config 5): a sample of replicas equals the
    single-lattice device chain with the same seed."""
    import supervillain_amd as sv
    R, N, sweeps = 128, 128, 6
    gens = [np.random.default_rng(r) for r in range(R)]
    B = VillainReplicas(R, N, 0.5, 2)
    B.cold()
    stats, obs = B.run(sweeps, gens, inline=True)
    phi, n = B.download()
    B.close()
    assert obs['WindingSquared'].shape == (R, sweeps) and np.isfinite(obs['ActionDensity']).all()
    for r in (0, 17, 127):
        L = sv.Lattice2D(N)
        S = sv.Villain(L, 0.5, 2)
        G = sv.generator.villain.NeighborhoodUpdate(S)
        G.rng = np.random.default_rng(r)
        cfg = G._steps(S.configurations(1)[0], sweeps)
        assert (np.asarray(cfg['phi'])[0] == phi[r]).all() and (np.asarray(cfg['n']) == n[r]).all()
        assert G.rng.bit_generator.state == gens[r].bit_generator.state
        assert G.accepted == stats['accepted'][r].sum()
        assert S.valid(cfg)


def test_one_shot_entry_point(oracle_lib):
    """sv_replicas_villain (SURVEY.md 8b's one-shot form over host arrays) == the oracle per replica."""
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import SvStats, rngs_from_numpy, rngs_to_numpy
    R, N, W, sweeps = 5, 16, 2, 4
    phi0, n0 = hot(R, N, W, 3)
    phi, n = phi0.copy(), n0.copy()
    gens = [np.random.default_rng(40 + r) for r in range(R)]
    r, addrs = rngs_from_numpy(gens)
    st = (SvStats * (R * sweeps))()
    obs = np.zeros((R, sweeps, 4))
    ctx = _native.context()
    ctx.check(_native.lib().sv_replicas_villain(ctx.handle, R, N, 0.4, W, float(np.pi), 1, _native.ptr(phi), _native.ptr(n),
                                                sweeps, r, st, _native.ptr(obs)), 'sv_replicas_villain')
    rngs_to_numpy(r, gens, addrs)
    for i in range(R):
        g = np.random.default_rng(40 + i)
        p, m = phi0[i].copy(), n0[i].copy()
        ref = oracle_lib.villain_neighborhood(N, 0.4, W, p, m, sweeps, g)
        assert (p == phi[i]).all() and (m == n[i]).all()
        assert g.bit_generator.state == gens[i].bit_generator.state
        assert [s.accepted for s in ref] == [st[i * sweeps + k].accepted for k in range(sweeps)]
        np.testing.assert_allclose(obs[i, -1, 0], offline(p, m)[0], rtol=1e-12)


@pytest.mark.parametrize('inline', [False, True])
def test_replicas_starting_on_a_buffered_half_word(oracle_lib, inline):
    """Replicas whose generators hold NumPy's buffered uint32 (has_uint32 = 1, as after an odd number of bounded
    draws or Lemire rejections) run the fast replica kernel's unpaired draw form; the others the paired one; every
    replica equals its own chain and, with inline observables, its offline measurement."""
    R, N, W, sweeps = 6, 64, 2, 4
    phi0, n0 = hot(R, N, W, 21)

    def gens_():
        gs = [np.random.default_rng(300 + r) for r in range(R)]
        for r in (1, 4):
            gs[r].integers(0, 3)  # leaves has_uint32 = 1
        return gs
    gens = gens_()
    assert gens[1].bit_generator.state['has_uint32'] == 1
    phi, n, stats, obs = run_batch(R, N, 0.5, W, phi0, n0, sweeps, gens, inline=inline)
    ref = gens_()
    for r in range(R):
        p, m = phi0[r].copy(), n0[r].copy()
        for s in range(sweeps):
            oracle_lib.villain_neighborhood(N, 0.5, W, p, m, 1, ref[r])
            if inline:
                act, w2, s0, s1 = offline(p, m)
                np.testing.assert_allclose(obs['ActionDensity'][r, s], 0.5 / 2 * act / (N * N), rtol=1e-12)
                assert obs['WindingSquared'][r, s] == w2 / (N * N)
                assert list(obs['TorusWrapping'][r, s]) == [s0, s1]
        assert (phi[r] == p).all() and (n[r] == m).all(), r
        assert gens[r].bit_generator.state == ref[r].bit_generator.state
