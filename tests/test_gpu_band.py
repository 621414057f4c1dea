"""Multi-sweep band launches (villain_sweep_hot_band) against the oracle.

Small periodic lattices (N <= 512, N % 8 == 0) run K consecutive hot sweeps per launch, one band of rows per XCD, each
sweep of a launch recomputing the deep-halo rows its successor reads (neighborhood.py:59-137 per sweep, every draw at
its global stream position).  The bar is the usual one: phi, n, the rng state and every sweep's accepted count
bit-exact, the acceptance sums within 1e-12 relative -- here per sweep, since each sweep of a band launch counts only
its bands' own rows.  Rejections forced inside a launch (at its first, a middle and its last sweep) exercise the
replay from the launch's scratch buffers.  The context's band counters show that the band kernel ran."""
import numpy as np
import pytest

from tests.golden import crafted_generator
from tests.test_gpu_overflow import single

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def bands_only():
    """Band launches only (the default prefers temporal blocks where they apply, tests/test_gpu_block.py)."""
    from supervillain_amd import _native
    ctx = _native.context()
    ctx.set_multisweep(2)
    try:
        yield
    finally:
        ctx.set_multisweep(0)


def check(N, kappa, W, phi0, n0, sweeps, make_gen, oracle_lib, band_expected=True):
    from supervillain_amd import _native
    ctx = _native.context()
    ctx.band_counts()
    gen = make_gen()
    phi, n, st, counts = single(N, kappa, W, phi0, n0, sweeps, gen)
    bands = ctx.band_counts()
    g = make_gen()
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood(N, kappa, W, p, m, sweeps, g)
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    assert [s.rejections for s in st] == [s.rejections for s in ref]
    np.testing.assert_allclose([s.acceptance_sum for s in st], [s.acceptance_sum for s in ref], rtol=1e-12)
    if band_expected:
        assert bands['sweeps'] > 0 and bands['launches'] > 0, (bands, counts)
    return ref, bands


def test_band_config2(oracle_lib):
    """Config 2 (L=256, kappa=0.5, W=1, cold start, seed 0): 40 sweeps in one call, per-sweep statistics."""
    N = 256
    zero = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    _, bands = check(N, 0.5, 1, *zero, 40, lambda: np.random.default_rng(0), oracle_lib)
    assert bands['sweeps'] >= 35


@pytest.mark.parametrize('N', [16, 24, 64, 136, 200, 256, 512])
def test_band_sizes(N, oracle_lib):
    """Band heights from 2 to 64 rows, column strips from 1 to 5 (512 may not fit a band's workgroups on one XCD:
    then it runs one sweep per launch), hot start, W = 2."""
    r = np.random.default_rng(N)
    phi0, n0 = r.uniform(-np.pi, np.pi, (N, N)), 2 * r.integers(-2, 3, (2, N, N)).astype(np.int64)
    check(N, 0.7, 2, phi0, n0, 23, lambda: np.random.default_rng(N + 1), oracle_lib, band_expected=N < 512)


@pytest.mark.parametrize('sweep,where', [(3, 0), (7, 1), (13, 2)])
def test_band_forced_rejection(sweep, where, oracle_lib):
    """A NumPy Lemire rejection forced into sweep 3 (a middle sweep of the first 7-sweep launch), 7 (the first
    sweep of the second) or 13 (its last), in a colour-0 or colour-1 choice block: the sweeps before it stand, the
    state before it comes from the launch's scratch buffer, the replay and the launches after it are exact."""
    N = 256
    V = N * N
    off = [V + V // 2 + 7, V + 3 * V // 2 + V // 2 + V // 4 + 3, 4 * V - 1][where]
    pos = 4 * V * sweep + off
    zero = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    ref, _ = check(N, 0.5, 1, *zero, 20, lambda: crafted_generator(sweep, pos, [0, 1, 1][where]), oracle_lib)
    assert sum(s.rejections for s in ref) >= 1
