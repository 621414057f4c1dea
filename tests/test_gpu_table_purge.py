"""The jump-table cache purge (VERDICT r3 lead (a)): one context sees more PCG64 increments than its table cache holds,
so it drops the cache while launches that hold its tables are queued -- deferred device-resident pipeline members
(each generator its own increment, no synchronization between them) and interleaved single-lattice chains.  The cache
is bounded to 2 increments for the test (sv_ctx_set_table_cap); every chain is compared with the CPU oracle or with
the host loop, and the purge counter proves the purges happened.  The purge drains the device before freeing
(capi.hip jump_tables), so no queued launch may read a freed table."""
import ctypes

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
from supervillain_amd.generator import villain as gv

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_cache():
    ctx = _native.context()
    ctx.set_table_cap(2)
    try:
        yield ctx
    finally:
        ctx.set_table_cap(0)


def test_interleaved_chains_vs_oracle(small_cache, oracle_lib):
    """Six NeighborhoodUpdate chains (six increments), stepped in turn through the C-ABI without synchronizing the
    device in between (each sweep batch is enqueued whole), against the oracle chain by chain."""
    ctx = small_cache
    Lib = _native.lib()
    N, kappa, W, rounds, per = 32, 0.5, 1, 4, 3
    seeds = list(range(40, 46))
    handles, states, gens = [], [], []
    try:
        for s in seeds:
            h = ctypes.c_void_p()
            ctx.check(Lib.sv_villain_create(ctx.handle, N, ctypes.byref(h)), 'sv_villain_create')
            handles.append(h)
            r = np.random.default_rng(s)
            phi = r.uniform(-np.pi, np.pi, (N, N))
            n = r.integers(-2, 3, (2, N, N)).astype(np.int64)
            states.append((phi.copy(), n.copy()))
            ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
            gens.append(np.random.default_rng(s + 1000))
        before = ctx.table_purges()
        accepted = [0] * len(seeds)
        for _ in range(rounds):
            for i, h in enumerate(handles):
                r = rng_from_numpy(gens[i])
                st = _native.stats_array(per)
                ctx.check(Lib.sv_villain_run(h, kappa, W, float(np.pi), 1, per, ctypes.byref(r), st, 2), 'run')
                rng_to_numpy(r, gens[i])
                accepted[i] += sum(st[k].accepted for k in range(per))
        assert ctx.table_purges() - before >= rounds * len(seeds) // 2
        for i, h in enumerate(handles):
            phi = np.empty((N, N))
            n = np.empty((2, N, N), dtype=np.int64)
            ctx.check(Lib.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'download')
            p, m = states[i]
            g = np.random.default_rng(seeds[i] + 1000)
            ref = oracle_lib.villain_neighborhood(N, kappa, W, p, m, rounds * per, g)
            assert (phi == p).all() and (n == m).all(), i
            assert gens[i].bit_generator.state == g.bit_generator.state
            assert accepted[i] == sum(s.accepted for s in ref)
    finally:
        for h in handles:
            Lib.sv_villain_destroy(h)


def test_deferred_hammer_across_purges(small_cache):
    """A device-resident Villain Hammer (five generators, five increments: the pipeline runs them deferred, one
    synchronization per step) with the cache dropped inside every step, against the per-step host loop."""
    ctx = small_cache
    S = sv.Villain(sv.Lattice2D(16), 0.4, 2)
    out = []
    for resident in (False, True):
        H = gv.Hammer(S)
        for G, s in zip(H.generators, [11, 12, 13, 14, 15]):
            G.rng = np.random.default_rng(s)
        before = ctx.table_purges()
        E = sv.Ensemble(S).generate(8, H, device_resident=resident)
        purges = ctx.table_purges() - before
        out.append((np.asarray(E.configuration.phi.array).copy(), np.asarray(E.configuration.n.array).copy(),
                    H.report(), [G.rng.bit_generator.state for G in H.generators if hasattr(G, 'rng')], purges))
    (p0, n0, r0, s0, _), (p1, n1, r1, s1, k1) = out
    assert k1 >= 8
    assert (p0 == p1).all() and (n0 == n1).all() and r0 == r1 and s0 == s1
