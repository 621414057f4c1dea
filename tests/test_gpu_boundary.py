"""The one-shot C-ABI entry points INTEGRATION.md section 2 tells a maintainer to bind, called through a
standalone ctypes binding written exactly as that section writes it (its own CDLL, sv_rng / sv_stats
structures, a fresh host copy of the fields per call), against the golden fixtures captured from the
reference (tools/make_golden.py):

  sv_villain_neighborhood  <- NeighborhoodUpdate.step   supervillain/generator/villain/neighborhood.py:59-137
  sv_worldline_coexact     <- CoexactUpdate.step        supervillain/generator/worldline/coexact.py:53-128
  sv_worldline_plaquette   <- PlaquetteUpdate.step      supervillain/generator/worldline/plaquette.py:35-104
"""
import ctypes
import os

import numpy as np
import pytest

from tests.golden import cases, generator_from, state_of

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'supervillain_amd', 'libsvhip.so')
_P = ctypes.POINTER


class _Rng(ctypes.Structure):  # sv_rng
    _fields_ = [('state_hi', ctypes.c_uint64), ('state_lo', ctypes.c_uint64),
                ('inc_hi', ctypes.c_uint64), ('inc_lo', ctypes.c_uint64),
                ('has_uint32', ctypes.c_int32), ('uinteger', ctypes.c_uint32)]


class _Stats(ctypes.Structure):  # sv_stats
    _fields_ = [('accepted', ctypes.c_int64), ('proposed', ctypes.c_int64),
                ('acceptance_sum', ctypes.c_double), ('rejections', ctypes.c_int64)]


@pytest.fixture(scope='module')
def binding():
    lib = ctypes.CDLL(LIB)
    lib.sv_ctx_create.argtypes = [ctypes.c_int, _P(ctypes.c_void_p)]
    lib.sv_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.sv_last_error.argtypes = [ctypes.c_void_p]
    lib.sv_last_error.restype = ctypes.c_char_p
    lib.sv_villain_neighborhood.argtypes = [
        ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_int64, ctypes.c_double, ctypes.c_int64,
        _P(ctypes.c_double), _P(ctypes.c_int64), ctypes.c_int32, _P(_Rng), _P(_Stats)]
    lib.sv_worldline_coexact.argtypes = [
        ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_int64, _P(ctypes.c_int64),
        ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _P(_Rng), _P(_Stats)]
    lib.sv_worldline_plaquette.argtypes = [
        ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_double, _P(ctypes.c_int64), ctypes.c_void_p,
        ctypes.c_int32, _P(ctypes.c_int64), _P(_Rng), _P(_Stats)]
    ctx = ctypes.c_void_p()
    assert lib.sv_ctx_create(int(os.environ.get('SV_DEVICE', '0')), ctypes.byref(ctx)) == 0
    yield lib, ctx
    lib.sv_ctx_destroy(ctx)


def to_rng(gen):
    s = gen.bit_generator.state
    st, inc = s['state']['state'], s['state']['inc']
    return _Rng(st >> 64, st & (2 ** 64 - 1), inc >> 64, inc & (2 ** 64 - 1), s['has_uint32'], s['uinteger'])


def from_rng(r, gen):
    s = gen.bit_generator.state
    s['state'] = {'state': (r.state_hi << 64) | r.state_lo, 'inc': (r.inc_hi << 64) | r.inc_lo}
    s['has_uint32'], s['uinteger'] = r.has_uint32, r.uinteger
    gen.bit_generator.state = s


def check(lib, ctx, rc):
    assert rc == 0, lib.sv_last_error(ctx).decode()


@pytest.mark.parametrize('fixture', ['villain_neighborhood.npz', 'villain_rejections.npz'])
def test_sv_villain_neighborhood_one_step_per_call(binding, fixture):
    """The INTEGRATION.md step(): one call per reference step, host arrays in and out."""
    lib, ctx = binding
    for c in cases(fixture):
        N, V = c['N'], c['N'] ** 2
        gen = generator_from(c['rng0'])
        phi = np.ascontiguousarray(c['phi0'], dtype=np.float64).copy()
        n = np.ascontiguousarray(c['n0'], dtype=np.int64).copy()
        for k in range(c['sweeps']):
            r, st = to_rng(gen), _Stats()
            check(lib, ctx, lib.sv_villain_neighborhood(
                ctx, N, c['kappa'], int(c['W']), c['interval_phi'], int(c['interval_n']),
                phi.ctypes.data_as(_P(ctypes.c_double)), n.ctypes.data_as(_P(ctypes.c_int64)), 1,
                ctypes.byref(r), ctypes.byref(st)))
            from_rng(r, gen)
            assert st.proposed == V and st.accepted == c['accepted'][k] - (c['accepted'][k - 1] if k else 0)
        assert (phi == c['phi']).all() and (n == c['n']).all(), (fixture, N)
        assert (state_of(gen) == c['rng1']).all()


def test_sv_villain_neighborhood_many_sweeps_per_call(binding):
    lib, ctx = binding
    for c in cases('villain_neighborhood.npz'):
        gen = generator_from(c['rng0'])
        phi = np.ascontiguousarray(c['phi0'], dtype=np.float64).copy()
        n = np.ascontiguousarray(c['n0'], dtype=np.int64).copy()
        r, st = to_rng(gen), (_Stats * c['sweeps'])()
        check(lib, ctx, lib.sv_villain_neighborhood(
            ctx, c['N'], c['kappa'], int(c['W']), c['interval_phi'], int(c['interval_n']),
            phi.ctypes.data_as(_P(ctypes.c_double)), n.ctypes.data_as(_P(ctypes.c_int64)), c['sweeps'],
            ctypes.byref(r), st))
        from_rng(r, gen)
        assert (phi == c['phi']).all() and (n == c['n']).all()
        assert (state_of(gen) == c['rng1']).all()
        assert list(np.cumsum([s.accepted for s in st])) == list(c['accepted'])


def test_sv_worldline_coexact_one_step_per_call(binding):
    lib, ctx = binding
    for c in cases('worldline_coexact.npz'):
        N = c['N']
        vf = not (c['W'] < float('inf'))
        v = np.ascontiguousarray(c['v'], dtype=np.float64 if vf else np.int64)
        m = np.zeros((2, N, N), dtype=np.int64)
        gen = generator_from(c['rng0'])
        for k in range(c['sweeps']):
            r, st = to_rng(gen), _Stats()
            check(lib, ctx, lib.sv_worldline_coexact(ctx, N, c['kappa'], c['W_eff'], int(c['interval_t']),
                                                     m.ctypes.data_as(_P(ctypes.c_int64)), v.ctypes.data, int(vf), 1,
                                                     ctypes.byref(r), ctypes.byref(st)))
            from_rng(r, gen)
            assert st.accepted == c['accepted'][k] - (c['accepted'][k - 1] if k else 0)
        assert (m == c['m']).all(), (N, c['W'])
        assert (state_of(gen) == c['rng1']).all()


def test_sv_worldline_plaquette_one_step_per_call(binding):
    """The reference's visit order is np.random.permutation(L.coordinates) (plaquette.py:63): the fixture
    records it per sweep as row-major site indices, which is what the entry point takes."""
    lib, ctx = binding
    for c in cases('worldline_plaquette.npz'):
        N = c['N']
        vf = not (c['W'] < float('inf'))
        m = np.zeros((2, N, N), dtype=np.int64)
        v = np.zeros((N, N), dtype=np.float64 if vf else np.int64)
        gen = generator_from(c['rng0'])
        for k in range(c['sweeps']):
            order = np.ascontiguousarray(c['order'][k], dtype=np.int64)
            r, st = to_rng(gen), _Stats()
            check(lib, ctx, lib.sv_worldline_plaquette(ctx, N, c['kappa'], c['W_eff'],
                                                       m.ctypes.data_as(_P(ctypes.c_int64)), v.ctypes.data, int(vf),
                                                       order.ctypes.data_as(_P(ctypes.c_int64)), ctypes.byref(r),
                                                       ctypes.byref(st)))
            from_rng(r, gen)
            assert st.accepted == c['accepted'][k] - (c['accepted'][k - 1] if k else 0), (N, k)
        assert (m == c['m']).all() and (v == c['v']).all(), (N, c['W'])
        assert (state_of(gen) == c['rng1']).all()


def test_errors_are_reported(binding):
    lib, ctx = binding
    phi = np.zeros((4, 4))
    n = np.zeros((2, 4, 4), dtype=np.int64)
    r, st = to_rng(np.random.default_rng(0)), _Stats()
    rc = lib.sv_villain_neighborhood(ctx, 1, 0.5, 1, np.pi, 1, phi.ctypes.data_as(_P(ctypes.c_double)),
                                     n.ctypes.data_as(_P(ctypes.c_int64)), 1, ctypes.byref(r), ctypes.byref(st))
    assert rc != 0 and lib.sv_last_error(ctx)
