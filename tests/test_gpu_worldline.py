"""CoexactUpdate and PlaquetteUpdate on the MI355X vs golden vectors and the CPU oracle."""
import numpy as np
import pytest

import supervillain_amd as sv
from tests.golden import cases, crafted_generator, generator_from, state_of

pytestmark = pytest.mark.gpu


def coexact_gpu(N, kappa, W, v, sweeps, gen, interval_t=1):
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, kappa, W)
    G = sv.generator.worldline.CoexactUpdate(S, interval_t=interval_t)
    G.rng = gen
    cfg = {'m': sv.Form(np.zeros((2, N, N), dtype=int), degree=1, lattice=L),
           'v': sv.Form(v.reshape(1, N, N), degree=2, lattice=L)}
    acc, accept = [], []
    for _ in range(sweeps):
        cfg = cfg | G.step(cfg)
        acc.append(G.accepted)
        accept.append(G.acceptance)
    return G, S, cfg, acc, accept


def test_coexact_golden():
    for c in cases('worldline_coexact.npz'):
        G, S, cfg, acc, accept = coexact_gpu(c['N'], c['kappa'], c['W'], c['v'], c['sweeps'],
                                             generator_from(c['rng0']), c['interval_t'])
        assert (np.asarray(cfg['m']) == c['m']).all(), (c['N'], c['W'])
        assert (state_of(G.rng) == c['rng1']).all()
        assert acc == list(c['accepted'])
        np.testing.assert_allclose(accept, c['acceptance'], rtol=1e-12)
        assert S.valid(cfg)
        assert np.asarray(cfg['m']).dtype == np.int64


@pytest.mark.parametrize('N,W', [(64, 1), (130, 3), (256, float('inf')), (63, 2)])
def test_coexact_oracle(N, W, oracle_lib):
    r = np.random.default_rng(N)
    v = r.integers(-3, 4, (N, N)) if W < float('inf') else r.standard_normal((N, N))
    G, S, cfg, acc, _ = coexact_gpu(N, 0.5, W, v, 5, np.random.default_rng(N + 1))
    m = np.zeros((2, N, N), dtype=np.int64)
    g = np.random.default_rng(N + 1)
    oracle_lib.worldline_coexact(N, 0.5, S._W, m, np.ascontiguousarray(v), 5, g)
    assert (np.asarray(cfg['m']) == m).all() and G.rng.bit_generator.state == g.bit_generator.state


def test_coexact_forced_rejection(oracle_lib):
    """interval_t=3 draws from 6 values, whose Lemire sampler can reject: force one."""
    N = 16
    V = N * N
    v = np.random.default_rng(3).integers(-3, 4, (N, N))
    for pos, half in [(V + 5, 0), (V + V // 4 + 2, 1)]:
        G, S, cfg, _, _ = coexact_gpu(N, 0.5, 1, v, 3, crafted_generator(pos, pos, half), interval_t=3)
        m = np.zeros((2, N, N), dtype=np.int64)
        g = crafted_generator(pos, pos, half)
        st = oracle_lib.worldline_coexact(N, 0.5, 1.0, m, np.ascontiguousarray(v), 3, g, interval_t=3)
        assert sum(s.rejections for s in st) >= 1
        assert (np.asarray(cfg['m']) == m).all() and G.rng.bit_generator.state == g.bit_generator.state


def test_plaquette_reference_order_golden():
    for c in cases('worldline_plaquette.npz'):
        N = c['N']
        L = sv.Lattice2D(N)
        S = sv.Worldline(L, c['kappa'], c['W'])
        G = sv.generator.worldline.PlaquetteUpdate(S)
        G.rng = generator_from(c['rng0'])
        cfg = S.configurations(1)[0]
        saved = np.random.get_state()
        np.random.seed(c['np_seed'])
        try:
            for k in range(c['sweeps']):
                cfg = cfg | G.step(cfg)
                assert G.accepted == c['accepted'][k]
                np.testing.assert_allclose(G.acceptance, c['acceptance'][k], rtol=1e-12)
        finally:
            np.random.set_state(saved)
        assert (np.asarray(cfg['m']) == c['m']).all() and (np.asarray(cfg['v'])[0] == c['v']).all()
        assert (state_of(G.rng) == c['rng1']).all()
        assert S.valid(cfg)


@pytest.mark.parametrize('N,W', [(32, 1), (64, 2), (100, float('inf'))])
def test_plaquette_reference_order_oracle(N, W, oracle_lib):
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.4, W)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(5)
    cfg = S.configurations(1)[0]
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.float64 if W == float('inf') else np.int64)
    g = np.random.default_rng(5)
    saved = np.random.get_state()
    np.random.seed(77)
    try:
        for sweep in range(3):
            st = np.random.get_state()
            o = np.random.permutation(L.coordinates)
            np.random.set_state(st)
            m0, v0, rng0 = m.copy(), v.copy(), state_of(g)
            cfg = cfg | G.step(cfg)
            s = oracle_lib.worldline_plaquette_seq(N, 0.4, S._W, m, v, (o[:, 0] % N) * N + (o[:, 1] % N), g)
            dm = int((np.asarray(cfg['m']) != m).sum())
            dv = int((np.asarray(cfg['v'])[0] != v).sum())
            if dm or dv:
                import os
                os.makedirs('gpurun_out', exist_ok=True)
                np.savez(f'gpurun_out/plaq_mismatch_{N}.npz', m0=m0, v0=v0, rng0=rng0, order=o,
                         m_gpu=np.asarray(cfg['m']), v_gpu=np.asarray(cfg['v'])[0], m_cpu=m, v_cpu=v)
            assert dm == 0 and dv == 0, (sweep, dm, dv, G.accepted, s.accepted)
            assert G.rng.bit_generator.state == g.bit_generator.state
    finally:
        np.random.set_state(saved)


def test_plaquette_reference_order_forced_rejection(oracle_lib):
    N = 12
    V = N * N
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.4, 1)
    pos, half = V // 2 + 9, 1  # inside the change_v block (choice over 3 values)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = crafted_generator(pos, pos, half)
    saved = np.random.get_state()
    np.random.seed(3)
    st0 = np.random.get_state()
    o = np.random.permutation(L.coordinates)
    np.random.set_state(st0)
    cfg = G.step(S.configurations(1)[0])
    np.random.set_state(saved)
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.int64)
    g = crafted_generator(pos, pos, half)
    st = oracle_lib.worldline_plaquette_seq(N, 0.4, 1.0, m, v, (o[:, 0] % N) * N + (o[:, 1] % N), g)
    assert st.rejections >= 1
    assert (np.asarray(cfg['m']) == m).all() and (np.asarray(cfg['v'])[0] == v).all()
    assert G.rng.bit_generator.state == g.bit_generator.state


@pytest.mark.parametrize('N,W', [(8, 1), (9, 2), (64, float('inf')), (256, 1)])
def test_plaquette_checkerboard_oracle(N, W, oracle_lib):
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.5, W)
    G = sv.generator.worldline.PlaquetteUpdate(S, mode='checkerboard')
    G.rng = np.random.default_rng(N)
    cfg = G._steps(S.configurations(1)[0], 6)
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.float64 if W == float('inf') else np.int64)
    g = np.random.default_rng(N)
    st = oracle_lib.worldline_plaquette_cb(N, 0.5, S._W, m, v, 6, g)
    assert (np.asarray(cfg['m']) == m).all() and (np.asarray(cfg['v'])[0] == v).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert G.accepted == sum(s.accepted for s in st)
    assert S.valid(cfg)


@pytest.mark.parametrize('N,W,sweeps', [(8, 1, 5), (9, 2, 4), (128, 1, 70), (64, float('inf'), 3)])
def test_plaquette_coexact_steps_oracle(N, W, sweeps, oracle_lib):
    """sv_worldline_plaquette_coexact_run: Sequentially(checkerboard Plaquette, Coexact) with one shared
    Generator, `sweeps` steps in one device call (crossing the 64-sweep batch at N=128), against the
    oracle run sweep by sweep in the same order."""
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
    vf = W == float('inf')
    Weff = 2 * np.pi if vf else float(W)
    r0 = np.random.default_rng(N + 1)
    v0 = (r0.uniform(-2, 2, (N, N)) if vf else r0.integers(-2, 3, (N, N))).astype(np.float64 if vf else np.int64)
    m0 = np.zeros((2, N, N), dtype=np.int64)
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, int(vf), ctypes.byref(h)), 'create')
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m0), _native.ptr(v0)), 'upload')
    gen = np.random.default_rng(7)
    r = rng_from_numpy(gen)
    st = _native.stats_array(2 * sweeps)
    ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, 0.5, Weff, 1, sweeps, ctypes.byref(r), st), 'run')
    rng_to_numpy(r, gen)
    m, v = np.empty_like(m0), np.empty_like(v0)
    ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    Lib.sv_worldline_destroy(h)
    g = np.random.default_rng(7)
    mm, vv = m0.copy(), v0.copy()
    for s in range(sweeps):
        sp = oracle_lib.worldline_plaquette_cb(N, 0.5, Weff, mm, vv, 1, g)[0]
        sc = oracle_lib.worldline_coexact(N, 0.5, Weff, mm, vv, 1, g)[0]
        assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
        np.testing.assert_allclose([st[2 * s].acceptance_sum, st[2 * s + 1].acceptance_sum],
                                   [sp.acceptance_sum, sc.acceptance_sum], rtol=1e-12)
    assert (m == mm).all() and (v == vv).all()
    assert gen.bit_generator.state == g.bit_generator.state


def _worldline_run(N, kappa, Weff, m0, v0, steps, gen, interval_t=1):
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, int(v0.dtype == np.float64), ctypes.byref(h)), 'create')
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m0), _native.ptr(v0)), 'upload')
    r = rng_from_numpy(gen)
    st = _native.stats_array(2 * steps)
    ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, kappa, Weff, interval_t, steps, ctypes.byref(r), st), 'run')
    rng_to_numpy(r, gen)
    m, v = np.empty_like(m0), np.empty_like(v0)
    ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    Lib.sv_worldline_destroy(h)
    return m, v, [st[i] for i in range(2 * steps)]


@pytest.mark.parametrize('start', ['cold', 'v_random'])
def test_config3_at_size(start, oracle_lib):
    """BASELINE config 3 at its own size: L=1024 Worldline, W=1, kappa=0.5, Plaquette (checkerboard) + Coexact
    per step, exactly as bench.py --workload worldline runs it (sv_worldline_plaquette_coexact_run), against the
    oracle step by step; from a cold start and from v ~ U{-3..3} (test_coexact_sparse.py:15-22 style)."""
    N, kappa, steps = 1024, 0.5, 4
    m0 = np.zeros((2, N, N), dtype=np.int64)
    v0 = (np.random.default_rng(11).integers(-3, 4, (N, N)) if start == 'v_random'
          else np.zeros((N, N))).astype(np.int64)
    gen = np.random.default_rng(0)
    m, v, st = _worldline_run(N, kappa, 1.0, m0, v0, steps, gen)
    g = np.random.default_rng(0)
    mm, vv = m0.copy(), v0.copy()
    for s in range(steps):
        sp = oracle_lib.worldline_plaquette_cb(N, kappa, 1.0, mm, vv, 1, g)[0]
        sc = oracle_lib.worldline_coexact(N, kappa, 1.0, mm, vv, 1, g)[0]
        assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
    assert (m == mm).all() and (v == vv).all()
    assert gen.bit_generator.state == g.bit_generator.state
    S = sv.Worldline(sv.Lattice2D(N), kappa, 1)
    assert S.valid({'m': sv.Form(m, degree=1, lattice=S.Lattice)})


def test_config3_reference_order_plaquette_at_size(oracle_lib):
    """The reference-order PlaquetteUpdate (plaquette.py:35-104, NumPy's global permutation) at config 3's size,
    one sweep after a Coexact sweep (so m != 0), against the sequential oracle."""
    N, kappa = 1024, 0.5
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, kappa, 1)
    C = sv.generator.worldline.CoexactUpdate(S)
    C.rng = np.random.default_rng(3)
    cfg = S.configurations(1)[0]
    cfg = cfg | C.step(cfg)
    m0 = np.asarray(cfg['m']).copy()
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(4)
    saved = np.random.get_state()
    np.random.seed(2024)
    try:
        st0 = np.random.get_state()
        o = np.random.permutation(L.coordinates)
        np.random.set_state(st0)
        cfg = cfg | G.step(cfg)
    finally:
        np.random.set_state(saved)
    m, v = m0.copy(), np.zeros((N, N), dtype=np.int64)
    g = np.random.default_rng(4)
    s = oracle_lib.worldline_plaquette_seq(N, kappa, 1.0, m, v, (o[:, 0] % N) * N + (o[:, 1] % N), g)
    assert (np.asarray(cfg['m']) == m).all() and (np.asarray(cfg['v'])[0] == v).all()
    assert G.accepted == s.accepted and G.rng.bit_generator.state == g.bit_generator.state


def _gpu_chain(N, kappa, W, mode, steps, seed):
    """Plaquette (checkerboard or reference order) + Coexact per step on the GPU from a cold start, through the
    C-ABI, fields resident on the device; the observables of tests/statparity.py per step."""
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy
    from tests.statparity import NAMES, observables
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.int64)
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'upload')
    r = rng_from_numpy(np.random.default_rng(seed))
    legacy = np.random.RandomState(seed + 1)  # the reference's global-RandomState permutation (plaquette.py:63)
    coords = np.array([(t, x) for t in range(N) for x in range(N)])
    st = _native.stats_array(1)
    out = np.empty((steps, len(NAMES)))
    try:
        for s in range(steps):
            if mode == 'checkerboard':
                ctx.check(Lib.sv_worldline_plaquette_checkerboard_run(h, kappa, W, 1, ctypes.byref(r), st), 'cb')
            else:
                o = legacy.permutation(coords)
                lin = np.ascontiguousarray((o[:, 0] % N) * N + o[:, 1] % N, dtype=np.int64)
                ctx.check(Lib.sv_worldline_plaquette_ordered_run(h, kappa, W, _native.ptr(lin), ctypes.byref(r), st),
                          'ordered')
            ctx.check(Lib.sv_worldline_coexact_run(h, kappa, W, 1, 1, ctypes.byref(r), st), 'coexact')
            ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
            out[s] = observables(m, v, kappa, W)
    finally:
        Lib.sv_worldline_destroy(h)
    return out


@pytest.mark.parametrize('N,steps', [(8, 20000), (16, 10000)])
def test_plaquette_checkerboard_statistical_parity(N, steps):
    """the checkerboard PlaquetteUpdate chain (the one config 3 benches) has the reference's
    stationary distribution.  Checkerboard Plaquette + Coexact against the golden-pinned reference-order
    Plaquette (plaquette.py:35-104) + Coexact, both on the GPU: blocked-bootstrap means of the Worldline action
    density and the per-direction (m - delta v / W)^2 agree within 4 standard errors
    (worldline-algorithm-comparison.py:38-95 is the reference's own template for such comparisons)."""
    from tests.statparity import NAMES, compare
    cb = _gpu_chain(N, 0.5, 1.0, 'checkerboard', steps, 1)
    ref = _gpu_chain(N, 0.5, 1.0, 'reference', steps, 2)
    zs = compare(cb, ref, steps // 20)
    for name, (z, ma, ea, mb, eb) in zs.items():
        assert abs(z) < 4.0, f'N={N} {name}: checkerboard {ma:.5f} +- {ea:.5f} vs reference order {mb:.5f} +- {eb:.5f}'
    assert all(0 < zs[n][2] < 0.01 for n in NAMES)


@pytest.mark.parametrize('N', [16, 256])
def test_plaquette_coexact_forced_rejection(N, oracle_lib):
    """A NumPy Lemire rejection forced into the change_v blocks of a combined Plaquette + Coexact run (the
    config-3 step, worldline_step_fused): in step 0's colour-0 block and in step 1's colour-1 block (raw u64
    positions: a step draws metropolis V, then four V/4-word bounded blocks, then Coexact V + 2 V/4).  The
    replayed step runs the fused kernel's GENERAL mode (skip lists); fields, statistics and the rng state
    match the oracle."""
    V = N * N
    per_step = 2 * V + V + V // 2
    for pos, half in [(V + V // 4 + 3, 0), (per_step + V + 3 * V // 4 + 1, 1)]:
        v0 = np.random.default_rng(5).integers(-2, 3, (N, N)).astype(np.int64)
        m0 = np.zeros((2, N, N), dtype=np.int64)
        gen = crafted_generator(pos, pos, half)
        m, v, st = _worldline_run(N, 0.5, 1.0, m0, v0, 3, gen)
        g = crafted_generator(pos, pos, half)
        mm, vv = m0.copy(), v0.copy()
        rej = 0
        for s in range(3):
            sp = oracle_lib.worldline_plaquette_cb(N, 0.5, 1.0, mm, vv, 1, g)[0]
            sc = oracle_lib.worldline_coexact(N, 0.5, 1.0, mm, vv, 1, g)[0]
            rej += sp.rejections + sc.rejections
            assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
            assert st[2 * s].rejections == sp.rejections, s
        assert rej >= 1
        assert (m == mm).all() and (v == vv).all()
        assert gen.bit_generator.state == g.bit_generator.state


def _ordered_run(N, kappa, m0, order, seed):
    """sv_worldline_plaquette_ordered_run through the C-ABI on (m0, v = 0); returns (rc, error, m, v, rng state)."""
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    try:
        m = np.ascontiguousarray(m0, dtype=np.int64).copy()
        v = np.zeros((N, N), dtype=np.int64)
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'upload')
        g = np.random.default_rng(seed)
        r = rng_from_numpy(g)
        st = _native.stats_array(1)
        o = np.ascontiguousarray(order, dtype=np.int64)
        rc = Lib.sv_worldline_plaquette_ordered_run(h, kappa, 1.0, _native.ptr(o), ctypes.byref(r), st)
        err = Lib.sv_last_error(ctx.handle).decode() if rc else ''
        if rc == 0:
            rng_to_numpy(r, g)
        ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
        return rc, err, m, v, g.bit_generator.state, st[0].accepted
    finally:
        Lib.sv_worldline_destroy(h)


@pytest.mark.parametrize('kind', ['row-major', 'column-major', 'reversed'])
def test_ordered_plaquette_deep_level_plans(kind, oracle_lib):
    """Visit orders far from random: row-major order chains every plaquette to its left and upper neighbours (2N - 1
    dependency levels, the device plan's relaxation runs 8 batches at N = 32), column-major likewise, reversed
    row-major too.  Bit-exact against the sequential oracle (plaquette.py:63-101 given the order)."""
    N, kappa = 32, 0.5
    lin = np.arange(N * N, dtype=np.int64)
    order = {'row-major': lin, 'column-major': (lin % N) * N + lin // N, 'reversed': lin[::-1].copy()}[kind]
    m0 = np.zeros((2, N, N), dtype=np.int64)
    rc, err, m, v, state, acc = _ordered_run(N, kappa, m0, order, 5)
    assert rc == 0, err
    mm, vv = m0.copy(), np.zeros((N, N), dtype=np.int64)
    g = np.random.default_rng(5)
    s = oracle_lib.worldline_plaquette_seq(N, kappa, 1.0, mm, vv, order, g)
    assert (m == mm).all() and (v == vv).all()
    assert state == g.bit_generator.state and acc == s.accepted


@pytest.mark.parametrize('bad', ['duplicate', 'out of range', 'negative'])
def test_ordered_plaquette_rejects_non_permutations(bad):
    """The reference draws its order as a permutation; anything else is refused (the device plan checks it) and the
    fields are left as they were."""
    N = 16
    order = np.arange(N * N, dtype=np.int64)
    if bad == 'duplicate':
        order[7] = order[3]
    elif bad == 'out of range':
        order[5] = N * N
    else:
        order[0] = -1
    m0 = np.random.default_rng(1).integers(-2, 3, (2, N, N))
    rc, err, m, v, _, _ = _ordered_run(N, 0.5, m0, order, 1)
    assert rc != 0 and 'permutation' in err
    assert (m == m0).all() and (v == 0).all()


@pytest.mark.parametrize('N,sweeps', [(16, 1), (48, 2), (64, 7)])
def test_reference_run_pipelined_sweeps(N, sweeps, oracle_lib):
    """Several reference-order sweeps in one call (sv_worldline_plaquette_reference_run, via PlaquetteUpdate._steps):
    the visit orders are drawn natively from the legacy global RandomState on host threads, pipelined with the device
    (sweep s + 2's draws and s + 1's swaps while s runs), and equal np.random.permutation's, sweep after sweep; the
    global state afterwards is NumPy's.  Against the sequential oracle fed NumPy's own permutations."""
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.45, 1)
    C = sv.generator.worldline.CoexactUpdate(S)
    C.rng = np.random.default_rng(12)
    cfg = S.configurations(1)[0]
    cfg = cfg | C.step(cfg)  # m != 0
    m = np.asarray(cfg['m']).copy()
    v = np.zeros((N, N), dtype=np.int64)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(13)
    saved = np.random.get_state()
    try:
        np.random.seed(31)
        cfg = cfg | G._steps(cfg, sweeps)
        after = np.random.get_state()
        np.random.seed(31)
        g = np.random.default_rng(13)
        acc = 0
        for _ in range(sweeps):
            o = np.random.permutation(L.coordinates)
            acc += oracle_lib.worldline_plaquette_seq(N, 0.45, 1.0, m, v, (o[:, 0] % N) * N + (o[:, 1] % N), g).accepted
        ref_after = np.random.get_state()
    finally:
        np.random.set_state(saved)
    assert (np.asarray(cfg['m']) == m).all() and (np.asarray(cfg['v'])[0] == v).all()
    assert G.accepted == acc and G.rng.bit_generator.state == g.bit_generator.state
    assert (after[1] == ref_after[1]).all() and after[2] == ref_after[2]


def test_reference_coexact_steps(oracle_lib):
    """Sequentially(PlaquetteUpdate [reference order], CoexactUpdate) on one Generator for 5 steps in one call
    (sv_worldline_plaquette_reference_coexact_run, what bench.py --plaquette reference times) against the oracle."""
    import ctypes
    from supervillain_amd import _native
    from supervillain_amd._abi import SvMT19937, rng_from_numpy, rng_to_numpy
    N, kappa, steps = 40, 0.5, 5
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.int64)
    legacy = np.random.RandomState(8)
    mt = SvMT19937()
    key = legacy.get_state()
    ctypes.memmove(mt.key, np.ascontiguousarray(key[1], dtype=np.uint32).ctypes.data, 624 * 4)
    mt.pos = int(key[2])
    gen = np.random.default_rng(21)
    try:
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'upload')
        r = rng_from_numpy(gen)
        st = _native.stats_array(2 * steps)
        ctx.check(Lib.sv_worldline_plaquette_reference_coexact_run(h, kappa, 1.0, 1, steps, ctypes.byref(mt),
                                                                   ctypes.byref(r), st), 'reference_coexact')
        rng_to_numpy(r, gen)
        ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    finally:
        Lib.sv_worldline_destroy(h)
    mm, vv = np.zeros((2, N, N), dtype=np.int64), np.zeros((N, N), dtype=np.int64)
    g = np.random.default_rng(21)
    lg = np.random.RandomState(8)
    for s in range(steps):
        o = lg.permutation(N * N).astype(np.int64)
        sp = oracle_lib.worldline_plaquette_seq(N, kappa, 1.0, mm, vv, o, g)
        sc = oracle_lib.worldline_coexact(N, kappa, 1.0, mm, vv, 1, g)[0]
        assert st[2 * s].accepted == sp.accepted and st[2 * s + 1].accepted == sc.accepted, s
    assert (m == mm).all() and (v == vv).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert (np.frombuffer(bytes(mt.key), dtype=np.uint32) == lg.get_state()[1]).all() and mt.pos == lg.get_state()[2]
