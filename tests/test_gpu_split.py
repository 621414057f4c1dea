"""The split replay (villain_sweep_hot_split) of a sweep that met a NumPy Lemire rejection, against the CPU oracle.

A rejected uint32 (neighborhood.py:105-107: NumPy's bounded sampler draws again) moves every later draw of its choice
block one half-word on; the replay runs each row with the descriptor of the block segment it lies in, fwd/bwd pairs
at opposite pairing parities included, and the strips whose rows straddle the switch on the skip-list body.  Forced
rejections (crafted PCG64 states) in each of the eight choice blocks, at the first rank (row 0: edge strips), the last
rank, interior ranks (one strip straddles, the rest run the split body) and a strip's first column, with the first
choice block starting on a whole word or on a buffered half-word: phi, n, the generator state and the counters must
equal the oracle's, and sv_ctx_split_counts proves the split kernel ran."""
import numpy as np
import pytest

import supervillain_amd as sv
from tests.golden import crafted_generator

pytestmark = pytest.mark.gpu


def hot(N, W, seed):
    r = np.random.default_rng(seed)
    return r.uniform(-np.pi, np.pi, (N, N)), W * r.integers(-2, 3, (2, N, N)).astype(np.int64)


def forced(seed, pos, half, has0):
    g = crafted_generator(seed, pos, half)
    if has0:  # the first choice block starts on a buffered half-word (uniform draws leave the buffer alone)
        st = g.bit_generator.state
        st['has_uint32'] = 1
        st['uinteger'] = 0x9E3779B9
        g.bit_generator.state = st
    return g


def word_of(N, c, j, rank, has0):
    """(u64 stream position in sweep 0, half) of the draw of rank `rank` in choice block j of colour c."""
    V = N * N
    q = rank - has0  # half-word index within the block's words (rank 0 with has0 = 1 is the buffered half)
    assert q >= 0
    return V + c * (V // 2 + V) + V // 2 + j * (V // 4) + q // 2, q % 2


def run(N, sweeps, gen, phi0, n0):
    L = sv.Lattice2D(N)
    S = sv.Villain(L, 0.5, 1)
    G = sv.generator.villain.NeighborhoodUpdate(S, path=2)
    G.rng = gen
    cfg = {'phi': sv.Form(phi0.reshape(1, N, N).copy(), degree=0, lattice=L),
           'n': sv.Form(n0.copy(), degree=1, lattice=L)}
    ctx = G._state()[0]
    ctx.sweep_counts()
    ctx.split_counts()
    cfg = G._steps(cfg, sweeps)
    return G, np.asarray(cfg['phi'])[0], np.asarray(cfg['n']), ctx.split_counts(), ctx.sweep_counts()


N = 1024
# ranks: the first (row 0, column 0: an edge strip), an interior rank (row 517), the first column of an interior strip
# (strip 3 starts at column 341), a rank in the last row, the last rank
RANKS = [0, (517 * N + 300) // 2, (600 * N + 341) // 2, (1023 * N + 700) // 2, N * N // 2 - 1]


@pytest.mark.parametrize('has0', [0, 1])
@pytest.mark.parametrize('blk', range(8))
def test_split_replay_each_block(blk, has0, oracle_lib):
    c, j = divmod(blk, 4)
    for i, rank in enumerate(RANKS):
        if has0 and rank == 0:
            continue  # (rank 0 draws the buffered half-word, not a fresh word)
        pos, half = word_of(N, c, j, rank, has0)
        seed = 1000 + 37 * blk + 5 * i + has0
        phi0, n0 = hot(N, 1, seed)
        G, phi, n, nsplit, counts = run(N, 2, forced(seed, pos, half, has0), phi0, n0)
        g = forced(seed, pos, half, has0)
        p, m = phi0.copy(), n0.copy()
        st = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, 2, g)
        assert sum(s.rejections for s in st) >= 1
        assert (phi == p).all() and (n == m).all(), (blk, rank, has0)
        assert G.rng.bit_generator.state == g.bit_generator.state
        assert G.accepted == sum(s.accepted for s in st)
        assert nsplit >= 1 and counts['fused'] == 0, (blk, rank, has0, nsplit, counts)


def test_split_replay_natural_rejections_4096(oracle_lib):
    """The bench-size lattice meets a natural rejection (seed 2024: in sweep 3) and replays it on the split kernel."""
    N4 = 4096
    phi0, n0 = np.zeros((N4, N4)), np.zeros((2, N4, N4), dtype=np.int64)
    G, phi, n, nsplit, counts = run(N4, 5, np.random.default_rng(2024), phi0, n0)
    g = np.random.default_rng(2024)
    st = oracle_lib.villain_neighborhood(N4, 0.5, 1, phi0, n0, 5, g)
    assert sum(s.rejections for s in st) >= 1
    assert (phi == phi0).all() and (n == n0).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert nsplit >= 1


@pytest.mark.parametrize('c,j', [(1, 3), (1, 2), (0, 3)])
def test_split_replay_straddler_in_a_head_slot(c, j, oracle_lib):
    """N = 2048 (663 strips: XCD ranges of 82 / 83): a rejection at row 300, column 517 makes straddling strips of which
    one already sits in a head slot that another is sent to; the slot permutation must still run every strip once
    (r5: the pairwise swaps ran one strip twice and left strip (rows 212-264, column strip 15) unswept)."""
    N2 = 2048
    V = N2 * N2
    rank = (300 * N2 + 517) // 2
    pos, half = V + c * (V // 2 + V) + V // 2 + j * (V // 4) + rank // 2, rank % 2
    seed = 600 + 4 * c + j
    r = np.random.default_rng(seed)
    phi0, n0 = r.uniform(-np.pi, np.pi, (N2, N2)), r.integers(-2, 3, (2, N2, N2)).astype(np.int64)
    G, phi, n, nsplit, counts = run(N2, 1, crafted_generator(seed, pos, half), phi0, n0)
    g = crafted_generator(seed, pos, half)
    st = oracle_lib.villain_neighborhood(N2, 0.5, 1, phi0, n0, 1, g)
    assert st[0].rejections == 1
    assert (phi == phi0).all() and (n == n0).all()
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert nsplit == 1 and counts['fused'] == 0


@pytest.mark.parametrize('N2', [2048, 4096])
def test_split_replay_random_positions(N2, oracle_lib):
    """Forced rejections at seeded random (colour, block, rank) on the lattices whose strip tables differ from N = 1024's
    (2048: 663 uniform strips; 4096: the per-XCD band schedule, 2992 strips): one sweep each, against the oracle."""
    V = N2 * N2
    pick = np.random.default_rng(N2)
    for i in range(4):
        c, j = int(pick.integers(0, 2)), int(pick.integers(0, 4))
        rank = int(pick.integers(1, V // 2))
        pos, half = V + c * (V // 2 + V) + V // 2 + j * (V // 4) + rank // 2, rank % 2
        seed = 900 + 10 * i + N2 // 1024
        r = np.random.default_rng(seed)
        phi0, n0 = r.uniform(-np.pi, np.pi, (N2, N2)), r.integers(-2, 3, (2, N2, N2)).astype(np.int64)
        G, phi, n, nsplit, counts = run(N2, 1, crafted_generator(seed, pos, half), phi0, n0)
        g = crafted_generator(seed, pos, half)
        st = oracle_lib.villain_neighborhood(N2, 0.5, 1, phi0, n0, 1, g)
        assert st[0].rejections == 1
        assert (phi == phi0).all() and (n == n0).all(), (N2, c, j, rank)
        assert G.rng.bit_generator.state == g.bit_generator.state
        assert nsplit == 1 and counts['fused'] == 0


PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645
M128 = (1 << 128) - 1


def crafted_two(seed, p1, half1, p2, half2):
    """A Generator(PCG64) whose raw outputs p1 < p2 (p2 - p1 odd) have their low (half=0) or high (half=1) 32 bits zero:
    two NumPy Lemire rejections in one sweep.  The state at output p1 is crafted as crafted_generator does; the
    increment is then solved for so that the state at p2 = A^d s1 + (sum_{i<d} A^i) inc takes the crafted form too
    (that sum is odd for odd d, so invertible mod 2^128; the free high word picks an odd increment)."""
    from tests.golden import _MINV
    d = p2 - p1
    assert d > 0 and d % 2 == 1
    out = {0: 0xDEADBEEF00000000, 1: 0x00000000DEADBEEF}
    h1 = (0x0123456789ABCDEF ^ (seed * 0x9E3779B1)) & ((1 << 58) - 1)
    s1 = (h1 << 64) | (h1 ^ out[half1])
    Ad, coef, a = 1, 0, 1
    for _ in range(d):
        coef = (coef + a) & M128
        a = (a * PCG_MULT) & M128
    Ad = a
    inv = pow(coef, -1, 1 << 128)
    for t in range(1 << 16):
        h2 = ((0x0FEDCBA987654321 ^ (seed * 0x85EBCA6B)) + t) & ((1 << 58) - 1)
        s2 = (h2 << 64) | (h2 ^ out[half2])
        inc = ((s2 - Ad * s1) * inv) & M128
        if inc & 1:
            break
    s = s1
    for _ in range(p1 + 1):
        s = ((s - inc) * _MINV) & M128
    g = np.random.default_rng(seed)
    st = g.bit_generator.state
    st['state']['state'] = s
    st['state']['inc'] = inc
    st['has_uint32'] = 0
    st['uinteger'] = 0
    g.bit_generator.state = st
    return g


@pytest.mark.parametrize('case', ['same row', 'different rows', 'both colours'])
def test_split_replay_two_rejections_in_one_sweep(case, oracle_lib):
    """split_plan takes up to two rejected words per sweep (one each in two choice blocks), and the replay
    switches descriptors per row for both.  Two crafted rejections in one sweep -- in two blocks of one colour on the
    same row, on different rows, and one in each colour -- replayed on the split kernel, against the oracle."""
    V = N * N
    (c1, j1, r1), (c2, j2, r2) = {
        'same row': ((0, 0, (517 * N + 300) // 2), (0, 2, (517 * N + 600) // 2)),
        'different rows': ((0, 1, (100 * N + 40) // 2), (0, 3, (700 * N + 900) // 2)),
        'both colours': ((0, 2, (333 * N + 123) // 2), (1, 1, (801 * N + 77) // 2)),
    }[case]
    p1, h1 = word_of(N, c1, j1, r1, 0)
    p2, h2 = word_of(N, c2, j2, r2, 0)
    if (p2 - p1) % 2 == 0:  # (the increment solve needs an odd distance: the next word of the same block)
        r2 += 2
        p2, h2 = word_of(N, c2, j2, r2, 0)
    seed = {'same row': 71, 'different rows': 72, 'both colours': 73}[case]
    phi0, n0 = hot(N, 1, seed)
    gen = crafted_two(seed, p1, h1, p2, h2)
    G, phi, n, nsplit, counts = run(N, 2, gen, phi0, n0)
    g = crafted_two(seed, p1, h1, p2, h2)
    p, m = phi0.copy(), n0.copy()
    st = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, 2, g)
    assert st[0].rejections == 2, [s.rejections for s in st]
    assert (phi == p).all() and (n == m).all(), case
    assert G.rng.bit_generator.state == g.bit_generator.state
    assert G.accepted == sum(s.accepted for s in st)
    assert nsplit >= 1 and counts['fused'] == 0, (case, nsplit, counts)
