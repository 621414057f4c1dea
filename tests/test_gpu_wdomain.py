"""Domain-decomposed Worldline steps (sv_domain_*_worldline) on the MI355X: any tile grid, emulated on one GPU
through the same halo pack/unpack path the RCCL ranks use (and the RCCL path itself through a one-rank
loopback), reproduces the single-lattice config-3 step (checkerboard PlaquetteUpdate + CoexactUpdate,
sv_worldline_plaquette_coexact_run) bit for bit -- against the CPU oracle and against the single-lattice fused
kernel at scale, including a forced NumPy Lemire rejection whose abort has to spread across tiles
("Worldline (config 3) decomposes the same way")."""
import ctypes

import numpy as np
import pytest

from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
from supervillain_amd.domain import WorldlineDomain, unique_id
from tests.golden import crafted_generator

pytestmark = pytest.mark.gpu


def start(N, seed):
    r = np.random.default_rng(seed)
    return np.zeros((2, N, N), dtype=np.int64), r.integers(-3, 4, (N, N)).astype(np.int64)


def run_domain(N, tiles, m0, v0, steps, gen, rccl=False, chunks=None):
    dom = WorldlineDomain(N, N, tiles, 0.5, 1, unique_id=unique_id() if rccl else None)
    try:
        dom.upload(m0, v0)
        st = []
        for k in (chunks or [steps]):
            st += dom.run(k, gen)
        m, v = dom.download()
    finally:
        dom.close()
    return m, v, st


def run_single(N, m0, v0, steps, gen):
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    try:
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m0), _native.ptr(v0)), 'upload')
        r = rng_from_numpy(gen)
        st = _native.stats_array(2 * steps)
        ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, 0.5, 1.0, 1, steps, ctypes.byref(r), st), 'run')
        rng_to_numpy(r, gen)
        m, v = np.empty_like(m0), np.empty_like(v0)
        ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    finally:
        Lib.sv_worldline_destroy(h)
    return m, v, [st[i] for i in range(2 * steps)]


def assert_same(a, b):
    (m, v, st, g), (mm, vv, stt, gg) = a, b
    assert (m == mm).all() and (v == vv).all()
    assert [s.accepted for s in st] == [s.accepted for s in stt]
    assert [s.rejections for s in st] == [s.rejections for s in stt]
    assert [s.acceptance_sum for s in st] == [s.acceptance_sum for s in stt]  # (exact sums, common.h)
    assert g.bit_generator.state == gg.bit_generator.state


@pytest.mark.parametrize('tiles', [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4)])
def test_oracle(tiles, oracle_lib):
    """N=24 (tiles down to 12 x 6: the ghost frame is 5 wide) against the oracle step by step."""
    N, steps = 24, 6
    m0, v0 = start(N, 3)
    g = np.random.default_rng(11)
    m, v, st = run_domain(N, tiles, m0, v0, steps, g)
    go = np.random.default_rng(11)
    mm, vv = m0.copy(), v0.copy()
    for s in range(steps):
        sp = oracle_lib.worldline_plaquette_cb(N, 0.5, 1.0, mm, vv, 1, go)[0]
        sc = oracle_lib.worldline_coexact(N, 0.5, 1.0, mm, vv, 1, go)[0]
        assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
        np.testing.assert_allclose([st[2 * s].acceptance_sum, st[2 * s + 1].acceptance_sum],
                                   [sp.acceptance_sum, sc.acceptance_sum], rtol=1e-12)
    assert (m == mm).all() and (v == vv).all()
    assert g.bit_generator.state == go.bit_generator.state


@pytest.mark.parametrize('N,tiles,steps', [(256, (2, 2), 5), (384, (2, 4), 4), (1024, (2, 4), 3)])
def test_equals_single_lattice(N, tiles, steps):
    """Larger lattices (interior and edge strips inside each tile) against the single-lattice fused step;
    N=1024 in 2 x 4 tiles is config 3 as 8 GPUs would run it."""
    m0, v0 = start(N, 7)
    a = run_domain(N, tiles, m0, v0, steps, g := np.random.default_rng(5)) + (g,)
    b = run_single(N, m0, v0, steps, gg := np.random.default_rng(5)) + (gg,)
    assert_same(a, b)


@pytest.mark.parametrize('tiles', [(2, 2), (1, 4)])
def test_forced_rejection(tiles, monkeypatch, oracle_lib):
    """A NumPy Lemire rejection forced into step 1's colour-1 change_v block: the tile that draws it aborts,
    the abort spreads through the halo messages, every tile replays from that step with the skip list
    (worldline_step_fused's GENERAL mode), in batches of 4 steps so the replay also crosses a batch."""
    monkeypatch.setenv('SV_DOMAIN_BATCH', '4')
    N, steps = 64, 6
    V = N * N
    per_step = 2 * V + V + V // 2
    pos = per_step + V + 3 * V // 4 + 5
    m0, v0 = start(N, 2)
    g = crafted_generator(pos, pos, 1)
    m, v, st = run_domain(N, tiles, m0, v0, steps, g)
    go = crafted_generator(pos, pos, 1)
    mm, vv = m0.copy(), v0.copy()
    rej = 0
    for s in range(steps):
        sp = oracle_lib.worldline_plaquette_cb(N, 0.5, 1.0, mm, vv, 1, go)[0]
        sc = oracle_lib.worldline_coexact(N, 0.5, 1.0, mm, vv, 1, go)[0]
        rej += sp.rejections
        assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
        assert st[2 * s].rejections == sp.rejections, s
    assert rej >= 1
    assert (m == mm).all() and (v == vv).all()
    assert g.bit_generator.state == go.bit_generator.state


def test_chunked_calls_continue_the_chain():
    """Several run() calls continue one chain (the tile ring's current buffer carries over)."""
    N = 128
    m0, v0 = start(N, 4)
    a = run_domain(N, (2, 2), m0, v0, 7, g := np.random.default_rng(8), chunks=[3, 1, 3]) + (g,)
    b = run_single(N, m0, v0, 7, gg := np.random.default_rng(8)) + (gg,)
    assert_same(a, b)


@pytest.mark.parametrize('N', [64, 512])
def test_rccl_loopback(N):
    """One rank, one tile, its halos through RCCL to itself: the exact RCCL send/recv code the 8-rank run
    uses, on one GPU."""
    m0, v0 = start(N, 9)
    a = run_domain(N, (1, 1), m0, v0, 4, g := np.random.default_rng(3), rccl=True) + (g,)
    b = run_single(N, m0, v0, 4, gg := np.random.default_rng(3)) + (gg,)
    assert_same(a, b)


def test_rectangular_lattice_decomposes_consistently():
    """An even rectangular Nt x Nx Worldline lattice (an engine extension: the reference's Lattice2D is square;
    bench.py's R1 runs one periodic tile of a decomposition this way) gives the same chain as one tile and as
    1 x 2 and 2 x 2 tiles."""
    Nt, Nx, steps = 64, 128, 4
    r = np.random.default_rng(6)
    m0, v0 = np.zeros((2, Nt, Nx), dtype=np.int64), r.integers(-3, 4, (Nt, Nx)).astype(np.int64)
    out = []
    for tiles in [(1, 1), (1, 2), (2, 2)]:
        dom = WorldlineDomain(Nt, Nx, tiles, 0.5, 1)
        try:
            dom.upload(m0, v0)
            g = np.random.default_rng(4)
            st = dom.run(steps, g)
            m, v = dom.download()
        finally:
            dom.close()
        out.append((m, v, st, g))
    for o in out[1:]:
        assert_same(o, out[0])
