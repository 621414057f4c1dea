"""The native legacy-RandomState permutation (sv_mt19937_permutation, host code of libsvhip.so) against NumPy's own
np.random.permutation and against the visit orders the reference drew itself (tests/golden/worldline_plaquette.npz,
captured from plaquette.py:63 by tools/make_golden.py).  CPU only: the entry point does no device work."""
import ctypes

import numpy as np
import pytest

from supervillain_amd import _native
from supervillain_amd._abi import SvMT19937, legacy_state_get, legacy_state_set
from tests.golden import cases


@pytest.fixture
def saved_legacy_state():
    st = np.random.get_state()
    yield
    np.random.set_state(st)


def native_permutation(mt, n):
    out = np.empty(n, dtype=np.int64)
    rc = _native.lib().sv_mt19937_permutation(ctypes.byref(mt), n, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


@pytest.mark.parametrize('seed,n,skip', [(0, 0, 0), (0, 1, 0), (0, 2, 0), (1, 10, 3), (7, 64, 623), (123, 1000, 1),
                                         (2 ** 32 - 1, 4096, 5), (5, 1 << 16, 0), (9, 65537, 200), (11, 1 << 20, 0)])
def test_equals_numpy_permutation(seed, n, skip, saved_legacy_state):
    """Sizes across mask boundaries (2^k, 2^k + 1), a fresh state, positions inside and at the end of a 624-word
    block; the permutation and the state afterwards (key, pos) equal NumPy's."""
    np.random.seed(seed)
    np.random.randint(0, 2 ** 31, size=skip)  # move the position inside the block
    mt, rest = legacy_state_get()
    ref = np.random.permutation(n)
    after = np.random.get_state()
    out = native_permutation(mt, n)
    assert (out == ref).all()
    legacy_state_set(mt, rest)
    st = np.random.get_state()
    assert (st[1] == after[1]).all() and st[2] == after[2] and st[3] == after[3]


def test_consecutive_permutations_and_2d_coordinates(saved_legacy_state):
    """plaquette.py:63 permutes the (V, 2) coordinate array: NumPy shuffles an index array, so the row-major image
    of the permuted coordinates is the index permutation itself -- over several consecutive sweeps."""
    np.random.seed(3)
    mt, _ = legacy_state_get()
    N = 8
    coords = np.stack(np.meshgrid(np.arange(N), np.arange(N), indexing='ij'), -1).reshape(-1, 2)
    for _ in range(5):
        ref = np.random.permutation(coords)
        assert ((ref[:, 0] % N) * N + (ref[:, 1] % N) == native_permutation(mt, N * N)).all()


def test_reference_golden_visit_orders():
    """The orders the reference itself drew (np.random.seed(np_seed), then one permutation per sweep)."""
    for c in cases('worldline_plaquette.npz'):
        mt = SvMT19937()
        st = np.random.RandomState(int(c['np_seed'])).get_state()
        ctypes.memmove(mt.key, np.ascontiguousarray(st[1], dtype=np.uint32).ctypes.data, 624 * 4)
        mt.pos = int(st[2])
        V = int(c['N']) ** 2
        for k in range(int(c['sweeps'])):
            assert (native_permutation(mt, V) == c['order'][k]).all(), (c['N'], k)


def test_bad_state_is_refused():
    mt = SvMT19937()
    mt.pos = 625
    out = np.empty(4, dtype=np.int64)
    assert _native.lib().sv_mt19937_permutation(ctypes.byref(mt), 4, out.ctypes.data_as(ctypes.c_void_p)) != 0
