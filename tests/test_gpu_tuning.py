"""Every runtime switch the library still reads (getenv "SV_*") changes scheduling only: a chain run under each one is
bit-for-bit the default run (fields, accepted counts, the NumPy bit-generator state, and -- since the float statistics
are exact sums (supervillain_amd/csrc/common.h) -- the acceptance sums and inline observables too, whatever the strip
heights or batch shapes), and the diagnostic switches print.

The switches are read per call, so they are set in-process (monkeypatch.setenv).  SV_DOMAIN_BATCH, SV_DOMAIN_DEPTH and
SV_DOMAIN_PREDICT are covered by test_gpu_domain.py / test_gpu_wdomain.py, SV_DEBUG_TIMING on domains there too."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.replicas import VillainReplicas

pytestmark = pytest.mark.gpu


def villain_chain(N, sweeps, seed=7, W=1):
    L = sv.Lattice2D(N)
    S = sv.Villain(L, 0.5, W)
    G = sv.generator.villain.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(seed)
    r = np.random.default_rng(seed + 1)
    cfg = {'phi': sv.Form(r.uniform(-np.pi, np.pi, (1, N, N)), degree=0, lattice=L),
           'n': sv.Form(W * r.integers(-2, 3, (2, N, N)).astype(np.int64), degree=1, lattice=L)}
    cfg = G._steps(cfg, sweeps)
    return np.asarray(cfg['phi']).copy(), np.asarray(cfg['n']).copy(), G.accepted, G.acceptance, \
        G.rng.bit_generator.state


def close(a, b):
    """bit for bit, floats included (the statistics do not depend on the launch geometry)"""
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and (a == b).all()


def same(a, b):
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
    assert a[2] == b[2] and a[4] == b[4]
    close(a[3], b[3])


@pytest.mark.parametrize('name,value,N', [
    ('SV_FUSED_TH', '9', 1024),             # strip height of the fused / hot kernels
    ('SV_STRIPS', '41x2,46', 1024),         # an explicit per-XCD strip schedule (8 bands of 128 rows)
    ('SV_STRIPS', 'uniform', 4096),         # uniform strips where band_strips is the default
    ('SV_BATCH', '3', 256),                 # sweeps per host round trip
    ('SV_BATCH', '1', 1024),
])
def test_villain_switch_is_result_neutral(monkeypatch, name, value, N):
    sweeps = 2 if N == 4096 else 8
    base = villain_chain(N, sweeps)
    monkeypatch.setenv(name, value)
    same(villain_chain(N, sweeps), base)


def test_batch_switch_takes_effect(monkeypatch, capfd):
    """SV_BATCH=3 plans 8 sweeps as 3 + 3 + 2 (SV_DEBUG_TIMING prints each plan)."""
    monkeypatch.setenv('SV_DEBUG_TIMING', '1')
    monkeypatch.setenv('SV_BATCH', '3')
    villain_chain(1024, 8)
    err = capfd.readouterr().err
    assert err.count('[sv] plan 3 sweeps') == 2 and err.count('[sv] plan 2 sweeps') == 1, err[-400:]


def replicas(R, N, sweeps):
    r = np.random.default_rng(3)
    phi0 = r.uniform(-np.pi, np.pi, (R, N, N))
    n0 = 2 * r.integers(-2, 3, (R, 2, N, N)).astype(np.int64)
    gens = [np.random.default_rng(50 + i) for i in range(R)]
    B = VillainReplicas(R, N, 0.5, 2)
    try:
        B.upload(phi0, n0)
        stats, obs = B.run(sweeps, gens, inline=True)
        phi, n = B.download()
    finally:
        B.close()
    return phi, n, stats, obs, [g.bit_generator.state for g in gens]


@pytest.mark.parametrize('name,value', [('SV_REP_CHUNK', '0'), ('SV_REP_CHUNK', '1'), ('SV_REP_CHUNK', '3'),
                                        ('SV_FUSED_TH', '13')])
def test_replica_switch_is_result_neutral(monkeypatch, name, value):
    base = replicas(24, 128, 20)
    monkeypatch.setenv(name, value)
    got = replicas(24, 128, 20)
    assert (got[0] == base[0]).all() and (got[1] == base[1]).all()
    for k in base[2]:
        close(got[2][k], base[2][k])
    for k in base[3]:
        close(got[3][k], base[3][k])
    assert got[4] == base[4]


def worldline(N, steps):
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    m0 = np.zeros((2, N, N), dtype=np.int64)
    v0 = np.random.default_rng(11).integers(-3, 4, (N, N)).astype(np.int64)
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    try:
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m0), _native.ptr(v0)), 'upload')
        gen = np.random.default_rng(0)
        r = rng_from_numpy(gen)
        st = _native.stats_array(2 * steps)
        ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, 0.5, 1.0, 1, steps, ctypes.byref(r), st), 'run')
        rng_to_numpy(r, gen)
        m, v = np.empty_like(m0), np.empty_like(v0)
        ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    finally:
        Lib.sv_worldline_destroy(h)
    return m, v, [(st[i].accepted, st[i].acceptance_sum) for i in range(2 * steps)], gen.bit_generator.state


@pytest.mark.parametrize('value', ['8', '12', '33'])
def test_worldline_strip_height_is_result_neutral(monkeypatch, value):
    """SV_WF_TH: rows per strip of worldline_step_fused (config 3's kernel)."""
    base = worldline(512, 3)
    monkeypatch.setenv('SV_WF_TH', value)
    got = worldline(512, 3)
    assert (got[0] == base[0]).all() and (got[1] == base[1]).all() and got[3] == base[3]
    close([a for a, _ in got[2]], [a for a, _ in base[2]])
    close([p for _, p in got[2]], [p for _, p in base[2]])


def test_alloc_log_prints(monkeypatch, capfd):
    """SV_ALLOC_LOG: every device allocation and free of the library is logged (fault attribution in suite runs)."""
    monkeypatch.setenv('SV_ALLOC_LOG', '1')
    villain_chain(64, 2)
    err = capfd.readouterr().err
    assert '[sv alloc] malloc' in err, err[-400:]
