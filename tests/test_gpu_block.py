"""Multi-sweep launches by temporal blocking (villain_sweep_block) against the oracle.

Small periodic lattices run K consecutive hot sweeps per launch; each workgroup keeps its block's deep-halo frame in
LDS for the whole launch (sweep j decides the block extended by 2(K-1-j) rows / columns above and left and 3(K-1-j)
below and right, neighborhood.py:59-137 per sweep, every draw at its global stream position) and never waits for
another.  The bar is the usual one: phi, n, the rng state and every sweep's accepted count and Lemire rejections
bit-exact, the acceptance sums within 1e-12 relative, per sweep.  Rejections forced inside a launch (its first, a
middle and its last sweep) exercise the replay from the launch's scratch buffers; the context's block counters show
that the kernel ran."""
import numpy as np
import pytest

from tests.golden import crafted_generator
from tests.test_gpu_overflow import single

pytestmark = pytest.mark.gpu


@pytest.fixture
def blocks_only():
    from supervillain_amd import _native
    ctx = _native.context()

    def use(K=0):
        ctx.set_multisweep(1, K)
    try:
        yield use
    finally:
        ctx.set_multisweep(0)


def check(N, kappa, W, phi0, n0, sweeps, make_gen, oracle_lib, interval_n=1, expected=True):
    from supervillain_amd import _native
    ctx = _native.context()
    ctx.block_counts()
    gen = make_gen()
    phi, n, st, counts = single(N, kappa, W, phi0, n0, sweeps, gen, interval_n=interval_n)
    blocks = ctx.block_counts()
    g = make_gen()
    p, m = phi0.copy(), n0.copy()
    ref = oracle_lib.villain_neighborhood(N, kappa, W, p, m, sweeps, g, interval_n=interval_n)
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert [s.accepted for s in st] == [s.accepted for s in ref]
    assert [s.rejections for s in st] == [s.rejections for s in ref]
    np.testing.assert_allclose([s.acceptance_sum for s in st], [s.acceptance_sum for s in ref], rtol=1e-12)
    if expected:
        assert blocks['sweeps'] > 0 and blocks['launches'] > 0, (blocks, counts)
    return ref, blocks


@pytest.mark.parametrize('K', [3, 5, 7])
def test_block_config2(K, blocks_only, oracle_lib):
    """Config 2 (L=256, kappa=0.5, W=1, cold start, seed 0): 40 sweeps in one call, K sweeps per launch."""
    blocks_only(K)
    N = 256
    zero = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    _, blocks = check(N, 0.5, 1, *zero, 40, lambda: np.random.default_rng(0), oracle_lib)
    assert blocks['sweeps'] >= 40 - 2 * K


def test_block_is_the_default_at_l256(oracle_lib):
    """Without a mode set, L=256 runs on the temporal blocks."""
    N = 256
    zero = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    check(N, 0.5, 1, *zero, 9, lambda: np.random.default_rng(5), oracle_lib)


@pytest.mark.parametrize('N', [24, 32, 64, 136, 200, 256, 512])
def test_block_sizes(N, blocks_only, oracle_lib):
    """Block sides 4 to 32 (N / 16, or the next divisor below), frames that wrap around the torus on every side,
    hot start, W = 2; N = 24 fits K = 3 only."""
    blocks_only(5)
    r = np.random.default_rng(N)
    phi0, n0 = r.uniform(-np.pi, np.pi, (N, N)), 2 * r.integers(-2, 3, (2, N, N)).astype(np.int64)
    check(N, 0.7, 2, phi0, n0, 23, lambda: np.random.default_rng(N + 1), oracle_lib)


def test_block_large_choices(blocks_only, oracle_lib):
    """W = 3, interval_n = 2 (five choices per link: Lemire's range 5), kappa = 0.3, L = 64."""
    blocks_only(3)
    N = 64
    r = np.random.default_rng(9)
    phi0, n0 = r.uniform(-np.pi, np.pi, (N, N)), 3 * r.integers(-3, 4, (2, N, N)).astype(np.int64)
    check(N, 0.3, 3, phi0, n0, 12, lambda: np.random.default_rng(10), oracle_lib, interval_n=2)


@pytest.mark.parametrize('sweep,where', [(3, 0), (7, 1), (14, 2), (15, 0)])
def test_block_forced_rejection(sweep, where, blocks_only, oracle_lib):
    """A NumPy Lemire rejection forced into sweep 3 (the first sweep of the second K = 3 launch), 7 (a middle sweep),
    14 (a last one) or 15 (a first one), in a colour-0 or colour-1 choice block: the sweeps before it stand,
    the state before it comes from the launch's scratch buffer, the replay and the launches after it are exact."""
    blocks_only(3)
    N = 256
    V = N * N
    off = [V + V // 2 + 7, V + 3 * V // 2 + V // 2 + V // 4 + 3, 4 * V - 1][where]
    pos = 4 * V * sweep + off
    zero = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    ref, _ = check(N, 0.5, 1, *zero, 20, lambda: crafted_generator(sweep, pos, [0, 1, 1][where]), oracle_lib)
    assert sum(s.rejections for s in ref) >= 1
