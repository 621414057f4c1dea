"""The headline kernel at the headline size against the oracle, and the n-range fallbacks of every Villain path.

villain_sweep_hot keeps n as int16 in LDS.  The reference keeps n as an unbounded int64
(generator/villain/neighborhood.py:103-107,128), so a state with |n| >= 2^14 -- or proposals W (index - interval_n)
too large for the int16 headroom -- must run on the general fused kernel's int32 image instead, on every path
(single lattice, domain tiles, replica batches), with the chain unchanged.  These tests start from n near the bound
at a tiny kappa (almost every proposal accepted: n random-walks across 2^14 within a sweep or two) and compare with
the CPU oracle bit for bit; the context's sweep counters show which kernel ran."""
import ctypes
import os

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
from supervillain_amd.domain import VillainDomain
from supervillain_amd.replicas import VillainReplicas

pytestmark = pytest.mark.gpu

B14 = 1 << 14


def single(N, kappa, W, phi0, n0, sweeps, gen, interval_n=1, path=2):
    """sv_villain_run through the C-ABI (as bench.py calls it); returns phi, n, per-sweep stats, sweep counts."""
    Lib = _native.lib()
    ctx = _native.context()
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, N, ctypes.byref(h)), 'sv_villain_create')
    try:
        phi = np.ascontiguousarray(phi0, dtype=np.float64).copy()
        n = np.ascontiguousarray(n0, dtype=np.int64).copy()
        ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
        ctx.sweep_counts()
        r = rng_from_numpy(gen)
        st = _native.stats_array(sweeps)
        ctx.check(Lib.sv_villain_run(h, kappa, W, float(np.pi), interval_n, sweeps, ctypes.byref(r), st, path),
                  'sv_villain_run')
        rng_to_numpy(r, gen)
        counts = ctx.sweep_counts()
        ctx.check(Lib.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'download')
    finally:
        Lib.sv_villain_destroy(h)
    return phi, n, [st[i] for i in range(sweeps)], counts


def test_headline_kernel_vs_oracle_at_L4096(oracle_lib):
    """BASELINE's headline workload exactly as bench.py runs it (L=4096, kappa=0.5, W=1, cold start, seed 0,
    sv_villain_run path 2 = villain_sweep_hot) for 5 sweeps, against the multi-core oracle bench.py times as its
    CPU baseline: phi, n, the rng state and the accepted counts bit-exact."""
    N, sweeps = 4096, 5
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    gen = np.random.default_rng(0)
    phi, n, st, counts = single(N, 0.5, 1, phi0, n0, sweeps, gen)
    assert counts['hot'] >= sweeps - 1 and counts['generic'] == 0, counts
    g = np.random.default_rng(0)
    threads = min(16, os.cpu_count() or 1)
    ref = oracle_lib.villain_neighborhood_mt(N, 0.5, 1, phi0, n0, sweeps, g, threads)
    assert (phi == phi0).all() and (n == n0).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    np.testing.assert_allclose([s.acceptance_sum for s in st], [s.acceptance_sum for s in ref], rtol=1e-12)


def near_bound(shape, seed):
    """n entries at +-(2^14 - 2): one or two accepted +-1 changes take a link across the int16 image's bound."""
    r = np.random.default_rng(seed)
    return (B14 - 2) * np.where(r.random(shape) < 0.5, 1, -1).astype(np.int64)


@pytest.mark.parametrize('mode', [3, 1])
def test_single_lattice_crosses_the_int16_bound(mode, oracle_lib):
    """One sweep per launch (mode 3): the int16 kernel until the sweep that meets |n| >= 2^14, the int32 one from
    there.  Temporal blocks (mode 1, the default at this size): their int32 LDS image takes the crossing in stride."""
    ctx = _native.context()
    ctx.set_multisweep(mode)
    try:
        N, kappa, sweeps = 64, 1e-9, 6
        phi0 = np.random.default_rng(1).uniform(-np.pi, np.pi, (N, N))
        n0 = near_bound((2, N, N), 2)
        ctx.block_counts()
        phi, n, st, counts = single(N, kappa, 1, phi0, n0, sweeps, np.random.default_rng(3))
        blocks = ctx.block_counts()
    finally:
        ctx.set_multisweep(0)
    g = np.random.default_rng(3)
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood(N, kappa, 1, p, m, sweeps, g)
    assert np.abs(m).max() >= B14  # the chain did cross the bound
    assert (phi == p).all() and (n == m).all()
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    if mode == 3:
        # the first sweep ran on the int16 kernel; from the sweep that met |n| >= 2^14 on, the int32 one
        assert counts['hot'] >= 1 and counts['fused'] >= 1 and counts['generic'] == 0, counts
    else:
        assert counts['hot'] == sweeps and blocks['sweeps'] == sweeps, (counts, blocks)


@pytest.mark.parametrize('W,interval_n', [(1, 20000), (4096, 3), (3, 2731)])
def test_large_proposals_bypass_the_int16_image(W, interval_n, oracle_lib):
    """|W| interval_n > 2^13: two accepted changes per sweep could carry a link past int16 from inside the bound
    (ADVICE r2), so these parameters never run on villain_sweep_hot; at kappa ~ 0 n moves by up to 2 |W| interval_n
    per sweep, against the oracle."""
    N, kappa, sweeps = 64, 1e-13, 3  # (dS ~ kappa (2 pi W interval_n)^2 must stay small)
    phi0 = np.zeros((N, N))
    n0 = np.zeros((2, N, N), dtype=np.int64)
    phi, n, st, counts = single(N, kappa, W, phi0, n0, sweeps, np.random.default_rng(5), interval_n=interval_n)
    g = np.random.default_rng(5)
    p, m = phi0.copy(), n0.copy()
    oracle_lib.villain_neighborhood(N, kappa, W, p, m, sweeps, g, interval_n=interval_n)
    assert np.abs(m).max() >= B14 or W * interval_n < B14
    assert (phi == p).all() and (n == m).all()
    assert counts['hot'] == 0 and counts['fused'] == sweeps, counts


def test_hot_bound_edge_stays_on_the_hot_kernel(oracle_lib):
    """|W| interval_n = 2^13 exactly is the largest the int16 image takes: hot kernel, equal to the oracle."""
    N, kappa, sweeps = 64, 1e-13, 3
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    phi, n, st, counts = single(N, kappa, 2, phi0, n0, sweeps, np.random.default_rng(6), interval_n=4096)
    g = np.random.default_rng(6)
    p, m = phi0.copy(), n0.copy()
    oracle_lib.villain_neighborhood(N, kappa, 2, p, m, sweeps, g, interval_n=4096)
    assert (phi == p).all() and (n == m).all()
    assert counts['hot'] >= 1, counts


@pytest.mark.parametrize('tiles', [(2, 4), (2, 2)])
def test_domain_crosses_the_int16_bound(tiles, oracle_lib):
    """Config 4's decomposition (deep halos, K = 4 sweeps per exchange): an OVERFLOW report replays the failing
    sweep on the int32 kernel on every tile instead of raising."""
    N, kappa, sweeps = 128, 1e-9, 7
    phi0 = np.random.default_rng(7).uniform(-np.pi, np.pi, (N, N))
    n0 = near_bound((2, N, N), 8)
    ctx = _native.context()
    dom = VillainDomain(N, N, tiles, kappa, 1)
    try:
        dom.upload(phi0, n0)
        ctx.sweep_counts()
        gen = np.random.default_rng(9)
        st = dom.run(sweeps, gen)
        counts = ctx.sweep_counts()
        phi, n = dom.download()
    finally:
        dom.close()
    g = np.random.default_rng(9)
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood(N, kappa, 1, p, m, sweeps, g)
    assert np.abs(m).max() >= B14
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    assert counts['hot'] >= 1 and counts['fused'] >= 1, counts


@pytest.mark.parametrize('inline', [False, True])
def test_replicas_cross_the_int16_bound(inline, oracle_lib):
    """Config 5's batch: replicas 1 and 3 start near the bound and move to the general kernel from their failing
    sweep on (split launches over replica maps); the others stay on villain_sweep_hot_fr.  Every replica equals its
    own oracle chain, and the inline observables their offline values."""
    from tests.test_gpu_replicas import offline
    R, N, kappa, sweeps = 4, 32, 1e-9, 5
    rr = np.random.default_rng(11)
    phi0 = rr.uniform(-np.pi, np.pi, (R, N, N))
    n0 = np.zeros((R, 2, N, N), dtype=np.int64)
    for r in (1, 3):
        n0[r] = near_bound((2, N, N), 20 + r)
    gens = [np.random.default_rng(200 + r) for r in range(R)]
    ctx = _native.context()
    B = VillainReplicas(R, N, kappa, 1)
    try:
        B.upload(phi0, n0)
        ctx.sweep_counts()
        stats, obs = B.run(sweeps, gens, inline=inline)
        counts = ctx.sweep_counts()
        phi, n = B.download()
    finally:
        B.close()
    assert counts['hot'] >= 1 and counts['fused'] >= 1, counts
    for r in range(R):
        g = np.random.default_rng(200 + r)
        p, m = phi0[r].copy(), n0[r].copy()
        for k in range(sweeps):
            s = oracle_lib.villain_neighborhood(N, kappa, 1, p, m, 1, g)
            assert stats['accepted'][r][k] == s[0].accepted
            if inline:
                act, w2, s0, s1 = offline(p, m)
                np.testing.assert_allclose(obs['ActionDensity'][r, k], kappa / 2 * act / (N * N), rtol=1e-12)
                assert obs['WindingSquared'][r, k] == w2 / (N * N)
                assert list(obs['TorusWrapping'][r, k]) == [s0, s1]
        if r in (1, 3):
            assert np.abs(m).max() >= B14
        assert (phi[r] == p).all() and (n[r] == m).all(), r
        assert gens[r].bit_generator.state == g.bit_generator.state


def test_inline_winding_with_large_plaquette_winding(oracle_lib):
    """dn up to ~6.4e4 inside the int16 image (n alternating +-16000 along each direction): dn^2 > 2^31, summed
    exactly by the fast replica kernel's WindingSquared (64-bit products)."""
    from tests.test_gpu_replicas import offline
    R, N, sweeps = 2, 32, 2
    t = np.arange(N)
    n0 = np.zeros((R, 2, N, N), dtype=np.int64)
    n0[:, 1] = np.where(t[:, None] % 2 == 0, 16000, -16000)  # n1 alternates along t
    n0[:, 0] = np.where(t[None, :] % 2 == 0, -16000, 16000)  # n0 alternates along x
    phi0 = np.zeros((R, N, N))
    gens = [np.random.default_rng(40 + r) for r in range(R)]
    ctx = _native.context()
    B = VillainReplicas(R, N, 0.3, 2)
    try:
        B.upload(phi0, n0)
        ctx.sweep_counts()
        stats, obs = B.run(sweeps, gens, inline=True)
        counts = ctx.sweep_counts()
    finally:
        B.close()
    assert counts['hot'] == sweeps, counts
    for r in range(R):
        g = np.random.default_rng(40 + r)
        p, m = phi0[r].copy(), n0[r].copy()
        for k in range(sweeps):
            oracle_lib.villain_neighborhood(N, 0.3, 2, p, m, 1, g)
            act, w2, s0, s1 = offline(p, m)
            assert w2 > 1 << 31
            assert obs['WindingSquared'][r, k] == w2 / (N * N)
            np.testing.assert_allclose(obs['ActionDensity'][r, k], 0.3 / 2 * act / (N * N), rtol=1e-12)
