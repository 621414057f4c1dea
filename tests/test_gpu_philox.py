"""The optional counter-based mode on the MI355X (sv_villain_run_philox, SURVEY.md 8(b) sv_rng mode 1): bit for bit
the oracle's Philox NeighborhoodUpdate chain (tests/test_philox.py ties that chain to the reference's distribution
and pins the generator to the published known answers), through the C-ABI and through the generator API."""
import ctypes

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd import _native
from supervillain_amd._abi import SvPhilox

pytestmark = pytest.mark.gpu


def start(N, W, seed):
    r = np.random.default_rng(seed)
    return r.uniform(-np.pi, np.pi, (N, N)), W * r.integers(-2, 3, (2, N, N)).astype(np.int64)


def device_run(N, kappa, W, phi, n, sweeps, key, counter, thr=0, interval_n=1):
    ctx = _native.context()
    L = _native.lib()
    h = ctypes.c_void_p()
    ctx.check(L.sv_villain_create(ctx.handle, N, ctypes.byref(h)), 'create')
    try:
        ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
        ph = SvPhilox(key, counter, thr)
        st = _native.stats_array(sweeps)
        rc = L.sv_villain_run_philox(h, kappa, W, float(np.pi), interval_n, sweeps, ctypes.byref(ph), st)
        if rc:
            return rc, None, None, None, None
        p, m = np.empty_like(phi), np.empty_like(n)
        ctx.check(L.sv_villain_download(h, _native.ptr(p), _native.ptr(m)), 'download')
        return 0, p, m, [st[i] for i in range(sweeps)], ph.counter
    finally:
        L.sv_villain_destroy(h)


@pytest.mark.parametrize('N,kappa,W,sweeps,counter', [(4, 0.5, 1, 5, 0), (16, 0.3, 2, 4, 7), (64, 0.8, 1, 3, (1 << 32) + 5),
                                                       (130, 0.5, 2, 2, 11), (256, 0.5, 1, 2, 123456789)])
def test_matches_oracle(N, kappa, W, sweeps, counter, oracle_lib):
    phi0, n0 = start(N, W, N)
    key = 0x0123456789ABCDEF ^ N
    rc, phi, n, st, c_end = device_run(N, kappa, W, phi0.copy(), n0.copy(), sweeps, key, counter)
    assert rc == 0 and c_end == counter + sweeps
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood_philox(N, kappa, W, p, m, sweeps, key, counter)
    assert (phi == p).all() and (n == m).all()
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    np.testing.assert_allclose([s.acceptance_sum for s in st], [s.acceptance_sum for s in ref], rtol=1e-12)


def test_redraws_match_oracle(oracle_lib):
    """A forced rejection threshold (half of all choice words redraw, several times over) through the device's
    in-place redraw loop."""
    N, W = 64, 2
    phi0, n0 = start(N, W, 5)
    rc, phi, n, st, _ = device_run(N, 0.5, W, phi0.copy(), n0.copy(), 3, 99, 0, thr=1 << 31)
    assert rc == 0
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood_philox(N, 0.5, W, p, m, 3, 99, 0, thr_override=1 << 31)
    assert (phi == p).all() and (n == m).all() and sum(s.rejections for s in ref) > 1000


def test_out_of_range_fails_loudly():
    N = 16
    phi0 = np.zeros((N, N))
    n0 = np.zeros((2, N, N), dtype=np.int64)
    n0[0, 3, 3] = 1 << 20  # beyond the int16 image
    rc, *_ = device_run(N, 0.5, 1, phi0, n0, 2, 1, 0)
    assert rc != 0
    rc, *_ = device_run(15, 0.5, 1, np.zeros((15, 15)), np.zeros((2, 15, 15), dtype=np.int64), 1, 1, 0)
    assert rc != 0  # odd N: the fused kernel only


def test_generator_api(oracle_lib):
    """NeighborhoodUpdate(..., philox=seed): step / KeepEvery / the resident Ensemble all follow the same counter."""
    N, kappa = 32, 0.5
    S = sv.Villain(sv.Lattice2D(N), kappa, 1)
    G = sv.generator.villain.NeighborhoodUpdate(S, philox=42)
    cfg = S.configurations(1)[0]
    for _ in range(3):
        cfg = G.step(cfg)
    assert G.philox_counter == 3 and G.sweeps == 3
    p, m = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    ref = oracle_lib.villain_neighborhood_philox(N, kappa, 1, p, m, 3, 42, 0)
    assert (np.asarray(cfg['phi'])[0] == p).all() and (np.asarray(cfg['n']) == m).all()
    assert G.accepted == sum(s.accepted for s in ref)
    out = []
    for resident in (False, True):
        H = sv.generator.villain.NeighborhoodUpdate(S, philox=7)
        E = sv.Ensemble(S).generate(5, sv.generator.KeepEvery(2, H), device_resident=resident)
        out.append((E.configuration.phi.array.copy(), E.configuration.n.array.copy(), H.philox_counter, H.report()))
    assert (out[0][0] == out[1][0]).all() and (out[0][1] == out[1][1]).all() and out[0][2:] == out[1][2:] == (10, out[0][3])
