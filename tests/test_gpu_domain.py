"""Domain-decomposed NeighborhoodUpdate (sv_domain_*) on the MI355X: any tile grid, emulated on one
GPU through the same halo pack/unpack path the RCCL ranks use, reproduces the single-lattice chain
bit-for-bit -- against the CPU oracle, the golden vectors from the reference, and the single-lattice
fused kernel at scale (including natural and forced NumPy Lemire rejections, whose abort has to
spread across tiles)."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.domain import VillainDomain, unique_id
from tests.golden import cases, crafted_generator, generator_from, state_of

pytestmark = pytest.mark.gpu


def hot(Nt, Nx, W, seed):
    r = np.random.default_rng(seed)
    return r.uniform(-np.pi, np.pi, (Nt, Nx)), W * r.integers(-2, 3, (2, Nt, Nx)).astype(np.int64)


def run_domain(Nt, Nx, tiles, kappa, W, phi0, n0, sweeps, gen, chunks=(None,), interval_phi=np.pi, interval_n=1,
               rccl=False, split=None):
    dom = VillainDomain(Nt, Nx, tiles, kappa, W, interval_phi, interval_n, unique_id=unique_id() if rccl else None)
    try:
        dom.upload(phi0, n0)
        dom.ctx.split_counts()  # (reset)
        stats = []
        left = sweeps
        for c in chunks:
            k = left if c is None else c
            stats += dom.run(k, gen)
            left -= k
        assert left == 0
        if split is not None:
            split.append(dom.ctx.split_counts())  # sweeps replayed on villain_sweep_hot_split (tile mode)
        phi, n = dom.download()
    finally:
        dom.close()
    return phi, n, stats


def assert_same(phi, n, st, gen, p, m, st_ref, g):
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == g.bit_generator.state
    assert [s.accepted for s in st] == [s.accepted for s in st_ref]
    np.testing.assert_allclose([s.acceptance_sum for s in st], [s.acceptance_sum for s in st_ref], rtol=1e-12)


GRIDS = [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (3, 2), (1, 8), (4, 4)]


@pytest.mark.parametrize('tiles', GRIDS)
def test_oracle_square(tiles, oracle_lib):
    N = 48
    phi0, n0 = hot(N, N, 2, 7)
    gen = np.random.default_rng(11)
    phi, n, st = run_domain(N, N, tiles, 0.4, 2, phi0, n0, 5, gen)
    g = np.random.default_rng(11)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.4, 2, p, m, 5, g)
    assert_same(phi, n, st, gen, p, m, st_ref, g)


@pytest.mark.parametrize('Nt,Nx,tiles', [(32, 96, (1, 3)), (32, 96, (2, 2)), (64, 16, (4, 1)), (256, 1024, (1, 2)),
                                         (260, 500, (2, 2))])
def test_oracle_rectangle(Nt, Nx, tiles, oracle_lib):
    """Rectangular lattices (the weak-scaling layouts 1x2 / 2x4 tiles of 4096^2 are rectangles):
    the oracle's natural extension of the reference's square-lattice chain."""
    phi0, n0 = hot(Nt, Nx, 1, Nt + Nx)
    gen = np.random.default_rng(Nt)
    phi, n, st = run_domain(Nt, Nx, tiles, 0.5, 1, phi0, n0, 3, gen)
    g = np.random.default_rng(Nt)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood_rect(Nt, Nx, 0.5, 1, p, m, 3, g)
    assert_same(phi, n, st, gen, p, m, st_ref, g)


@pytest.mark.parametrize('fixture', ['villain_neighborhood.npz', 'villain_rejections.npz'])
def test_golden(fixture):
    """The reference's own chains (even N), decomposed into 2 x 2 tiles where they are big enough."""
    ran = 0
    for c in cases(fixture):
        N = c['N']
        if N % 2 or N < 4:
            continue
        tiles = (2, 2) if N % 4 == 0 and N >= 8 else (1, 1)
        gen = generator_from(c['rng0'])
        phi, n, st = run_domain(N, N, tiles, c['kappa'], c['W'], c['phi0'], c['n0'].reshape(2, N, N), c['sweeps'], gen,
                                interval_phi=c['interval_phi'], interval_n=c['interval_n'])
        assert (phi == c['phi'].reshape(N, N)).all() and (n == c['n'].reshape(2, N, N)).all(), (fixture, N)
        assert (state_of(gen) == c['rng1']).all()
        assert list(np.cumsum([s.accepted for s in st])) == list(c['accepted'])
        ran += 1
    assert ran > 0


@pytest.mark.parametrize('batch', ['', '1', '2'])
@pytest.mark.parametrize('tiles', [(2, 2), (1, 8), (4, 4), (2, 4)])
def test_forced_rejections(tiles, batch, oracle_lib, monkeypatch):
    """Rejections placed in different blocks (and so in different tiles); the abort must reach every
    tile before its ring buffer is overwritten.  batch: SV_DOMAIN_BATCH (the adaptive batch of a large
    lattice is a few sweeps: aborts then land on batch boundaries)."""
    if batch:
        monkeypatch.setenv('SV_DOMAIN_BATCH', batch)
    N = 128
    V = N * N
    for pos, half in [(V + V // 2 + 7, 0), (V + V // 2 + V // 4 + 3, 1), (4 * V - 1, 1), (4 * V + V + V // 2 + 11, 0),
                      (2 * V + 5, 0)]:
        phi0, n0 = hot(N, N, 1, pos)
        gen = crafted_generator(pos % 1000, pos, half)
        phi, n, st = run_domain(N, N, tiles, 0.3, 1, phi0, n0, 3, gen)
        g = crafted_generator(pos % 1000, pos, half)
        p, m = phi0.copy(), n0.copy()
        st_ref = oracle_lib.villain_neighborhood(N, 0.3, 1, p, m, 3, g)
        assert sum(s.rejections for s in st_ref) >= 1
        assert_same(phi, n, st, gen, p, m, st_ref, g)
        assert [s.rejections for s in st] == [s.rejections for s in st_ref]


@pytest.mark.parametrize('depth', ['1', '2', '3', '5', '8'])
@pytest.mark.parametrize('tiles', [(2, 2), (1, 4), (2, 4)])
def test_deep_halo_depths(depth, tiles, oracle_lib, monkeypatch):
    """K sweeps per halo exchange (SV_DOMAIN_DEPTH; the default is 4): every depth, with groups cut short by the
    call's sweep count (11 = 2K + 3 at K = 4) and a forced NumPy Lemire rejection whose abort spreads one tile-hop
    per exchange, equals the oracle's single-lattice chain."""
    monkeypatch.setenv('SV_DOMAIN_DEPTH', depth)
    N = 128
    V = N * N
    pos, half = 4 * V + V + V // 2 + 11, 0  # sweep 1, a colour-0 choice block
    phi0, n0 = hot(N, N, 1, 99)
    gen = crafted_generator(5, pos, half)
    split = []
    phi, n, st = run_domain(N, N, tiles, 0.45, 1, phi0, n0, 11, gen, split=split)
    g = crafted_generator(5, pos, half)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.45, 1, p, m, 11, g)
    assert sum(s.rejections for s in st_ref) >= 1
    assert_same(phi, n, st, gen, p, m, st_ref, g)
    assert [s.rejections for s in st] == [s.rejections for s in st_ref]
    # the replay of the failing sweep ran on the split kernel in tile mode, at depth 1 and at the deeper frames of
    # the K > 1 groups (shifted region origins) alike
    assert split[0] >= 1, split


@pytest.mark.parametrize('tiles', [(2, 2), (2, 4)])
@pytest.mark.parametrize('pos_half', [(8 * 128 * 128 + 3 * 128 * 128 // 2 + 7, 0), (12 * 128 * 128 + 3 * 128 * 128 + 5, 1),
                                      (16 * 128 * 128 + 2 * 128 * 128 + 128 * 128 // 4 - 1, 1)])
def test_predicted_rejections(tiles, pos_half, oracle_lib, monkeypatch, capfd):
    """Rejection prediction: the words of the next batch are scanned while a batch runs, so a NumPy Lemire rejection
    in sweep 2, 3 or 4 (a colour-0 choice block, a colour-1 one, the last word of a colour-0 block) becomes a skip
    list before its batch is planned and nothing aborts; the chain equals the oracle's."""
    monkeypatch.setenv('SV_DOMAIN_BATCH', '2')
    monkeypatch.setenv('SV_DOMAIN_PREDICT', '1')  # (on by default only with several RCCL ranks)
    monkeypatch.setenv('SV_DEBUG_TIMING', '1')
    N = 128
    pos, half = pos_half
    phi0, n0 = hot(N, N, 1, 5)
    gen = crafted_generator(3, pos, half)
    phi, n, st = run_domain(N, N, tiles, 0.4, 1, phi0, n0, 7, gen)
    g = crafted_generator(3, pos, half)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.4, 1, p, m, 7, g)
    assert sum(s.rejections for s in st_ref) >= 1
    assert_same(phi, n, st, gen, p, m, st_ref, g)
    assert [s.rejections for s in st] == [s.rejections for s in st_ref]
    err = capfd.readouterr().err
    assert '[sv domain] 7 sweeps' in err and 'aborts 0' in err, err


@pytest.mark.parametrize('interval_n,W,depth', [(2, 1, '4'), (6, 2, '3'), (6, 1, '8')])
def test_predicted_rejections_other_choice_counts(interval_n, W, depth, oracle_lib, monkeypatch, capfd):
    """Choice over 5 or 13 values (NumPy thresholds 1 and 9), W = 2, depths 3 / 4 / 8: a forced rejection in sweep 3
    is predicted (no abort) and the decomposed chain equals the oracle's."""
    monkeypatch.setenv('SV_DOMAIN_BATCH', '2')
    monkeypatch.setenv('SV_DOMAIN_PREDICT', '1')
    monkeypatch.setenv('SV_DOMAIN_DEPTH', depth)
    monkeypatch.setenv('SV_DEBUG_TIMING', '1')
    N = 128
    V = N * N
    pos = 12 * V + 3 * V + V // 3
    phi0, n0 = hot(N, N, W, 17)
    gen = crafted_generator(11, pos, 1)
    phi, n, st = run_domain(N, N, (2, 4), 0.35, W, phi0, n0, 6, gen, interval_n=interval_n)
    g = crafted_generator(11, pos, 1)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.35, W, p, m, 6, g, interval_n=interval_n)
    assert sum(s.rejections for s in st_ref) >= 1
    assert_same(phi, n, st, gen, p, m, st_ref, g)
    assert [s.rejections for s in st] == [s.rejections for s in st_ref]
    err = capfd.readouterr().err
    assert '[sv domain] 6 sweeps' in err and 'aborts 0' in err, err


@pytest.mark.parametrize('tiles', [(2, 4), (2, 2), (1, 8)])
def test_prediction_partitioned_over_tiles(tiles, oracle_lib, monkeypatch, capfd):
    """The rejection scan split into one part per tile -- the partition several RCCL ranks use, each scanning its
    share into its own batch summary -- and the merge of every summary's finds into the next batch's skip lists.
    interval_n = 125576 gives NumPy's Lemire sampler the threshold 250996 (~4 rejected words per N=128 sweep, ~2 per
    part and batch of 4 sweeps).  The call's first batch is scanned in front of it (no scan ran ahead of it), every
    later one behind its predecessor; no batch may abort, and the chain equals the oracle's."""
    monkeypatch.setenv('SV_DOMAIN_BATCH', '4')
    monkeypatch.setenv('SV_DOMAIN_PREDICT', '1')
    monkeypatch.setenv('SV_DEBUG_TIMING', '1')
    N, sweeps, interval_n = 128, 16, 125576
    phi0, n0 = hot(N, N, 1, 31)
    gen = np.random.default_rng(12)
    phi, n, st = run_domain(N, N, tiles, 0.5, 1, phi0, n0, sweeps, gen, interval_n=interval_n)
    g = np.random.default_rng(12)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, sweeps, g, interval_n=interval_n)
    assert sum(s.rejections for s in st_ref) >= 2 * sweeps
    assert_same(phi, n, st, gen, p, m, st_ref, g)
    assert [s.rejections for s in st] == [s.rejections for s in st_ref]
    err = capfd.readouterr().err
    line = [x for x in err.splitlines() if x.startswith(f'[sv domain] {sweeps} sweeps')]
    assert line and 'predicted batches 4 (1 pre-scanned), aborts 0' in line[0], err


def test_prediction_not_reused_across_interval_n(oracle_lib, monkeypatch):
    """A scan kept for the batch the next call starts with is tied to the draw parameters it tested: a next call
    with another interval_n (other Lemire threshold) must not take its finds as skip positions."""
    monkeypatch.setenv('SV_DOMAIN_PREDICT', '1')
    monkeypatch.setenv('SV_DOMAIN_BATCH', '2')
    N = 128
    phi0, n0 = hot(N, N, 1, 41)
    dom_gen = np.random.default_rng(13)
    dom = VillainDomain(N, N, (2, 2), 0.5, 1, interval_n=1048064)
    try:
        dom.upload(phi0, n0)
        dom.run(2, dom_gen)  # leaves a scan for the next call's first batch (threshold 2095104)
        dom.interval_n = 1
        st = dom.run(2, dom_gen)  # threshold 1: those words are not rejected
        phi, n = dom.download()
    finally:
        dom.close()
    g = np.random.default_rng(13)
    p, m = phi0.copy(), n0.copy()
    oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, 2, g, interval_n=1048064)
    ref = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, 2, g, interval_n=1)
    assert_same(phi, n, st, dom_gen, p, m, ref, g)


def test_chunked_calls_continue_the_chain(oracle_lib):
    """Calls of 3 + 1 + 4 sweeps (ring index carried across calls) equal one call of 8."""
    N = 64
    phi0, n0 = hot(N, N, 1, 3)
    gen = np.random.default_rng(5)
    phi, n, st = run_domain(N, N, (2, 4), 0.6, 1, phi0, n0, 8, gen, chunks=(3, 1, 4))
    g = np.random.default_rng(5)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.6, 1, p, m, 8, g)
    assert_same(phi, n, st, gen, p, m, st_ref, g)


def single_lattice(N, kappa, W, phi0, n0, sweeps, gen):
    L = sv.Lattice2D(N)
    G = sv.generator.villain.NeighborhoodUpdate(sv.Villain(L, kappa, W), path=2)
    G.rng = gen
    cfg = {'phi': sv.Form(phi0.reshape(1, N, N).copy(), degree=0, lattice=L),
           'n': sv.Form(n0.copy(), degree=1, lattice=L)}
    cfg = G._steps(cfg, sweeps)
    return np.asarray(cfg['phi'])[0], np.asarray(cfg['n']), G


def exact_acceptance(st, V):
    """NeighborhoodUpdate.acceptance folded from these statistics the way the generator folds them"""
    acc = 0.
    for s in st:
        acc += s.acceptance_sum / V
    return acc


@pytest.mark.parametrize('tiles', [(2, 4), (1, 8)])
def test_equals_single_lattice_at_scale(tiles):
    """L=1024 (interior strips take the fast draw path): decomposed == single-lattice fused kernel."""
    N = 1024
    phi0, n0 = hot(N, N, 1, 21)
    gen = np.random.default_rng(8)
    phi, n, st = run_domain(N, N, tiles, 0.5, 1, phi0, n0, 4, gen)
    p, m, G = single_lattice(N, 0.5, 1, phi0, n0, 4, np.random.default_rng(8))
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == G.rng.bit_generator.state
    assert sum(s.accepted for s in st) == G.accepted
    assert exact_acceptance(st, N * N) == G.acceptance  # (exact sums: the tile grid cannot enter them)


@pytest.mark.parametrize('batch', ['', '5', 'predict'])
def test_natural_rejections_bench_size(batch, monkeypatch):
    """L=4096 in 2 x 4 tiles for 96 sweeps: NumPy rejects ~1.6% of sweeps' draws somewhere, so the
    abort / replay protocol runs on real data; the chain equals the single-lattice one.  batch: as above."""
    if batch == 'predict':
        monkeypatch.setenv('SV_DOMAIN_PREDICT', '1')  # the first batch aborts at sweep 3, later ones are predicted
    elif batch:
        monkeypatch.setenv('SV_DOMAIN_BATCH', batch)
    N = 4096
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    gen = np.random.default_rng(2024)
    phi, n, st = run_domain(N, N, (2, 4), 0.5, 1, phi0, n0, 96, gen)
    p, m, G = single_lattice(N, 0.5, 1, phi0, n0, 96, np.random.default_rng(2024))
    assert sum(s.rejections for s in st) >= 1  # seed 2024 meets NumPy rejections in sweeps 3 and 89
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == G.rng.bit_generator.state
    assert sum(s.accepted for s in st) == G.accepted
    assert exact_acceptance(st, N * N) == G.acceptance  # (exact sums: the tile grid cannot enter them)


@pytest.mark.parametrize('tiles', [(1, 2), (2, 1)])
def test_two_rank_layouts_at_scale(tiles):
    """The N = 2 layouts of L=4096 (tiles of 4096 x 2048 / 2048 x 4096, 37-row strips over ~1.8 rounds of the chip's
    workgroup slots) in tile emulation: the chain equals the single lattice's (which runs its descending strip
    table), through a NumPy rejection (seed 2024, sweep 3)."""
    N = 4096
    phi0, n0 = np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    gen = np.random.default_rng(2024)
    phi, n, st = run_domain(N, N, tiles, 0.5, 1, phi0, n0, 12, gen)
    p, m, G = single_lattice(N, 0.5, 1, phi0, n0, 12, np.random.default_rng(2024))
    assert sum(s.rejections for s in st) >= 1
    assert (phi == p).all() and (n == m).all()
    assert gen.bit_generator.state == G.rng.bit_generator.state
    assert sum(s.accepted for s in st) == G.accepted
    assert exact_acceptance(st, N * N) == G.acceptance  # (exact sums: the tile grid cannot enter them)


@pytest.mark.parametrize('predict', ['0', '1'])
@pytest.mark.parametrize('N,sweeps', [(64, 5), (1024, 3), (256, 40)])
def test_rccl_loopback(N, sweeps, predict, oracle_lib, monkeypatch):
    """One rank, one tile, every halo message through ncclSend/ncclRecv to itself and the batch
    summary (with the rejection scan's words) through ncclAllGather: the RCCL code path of the multi-GPU run, on one
    GPU; N=256 over 40 sweeps in batches of 8 runs predicted batches."""
    monkeypatch.setenv('SV_DOMAIN_PREDICT', predict)
    if N == 256:
        monkeypatch.setenv('SV_DOMAIN_BATCH', '8')
    phi0, n0 = hot(N, N, 1, N)
    gen = np.random.default_rng(N)
    phi, n, st = run_domain(N, N, (1, 1), 0.5, 1, phi0, n0, sweeps, gen, rccl=True)
    g = np.random.default_rng(N)
    p, m = phi0.copy(), n0.copy()
    st_ref = oracle_lib.villain_neighborhood(N, 0.5, 1, p, m, sweeps, g)
    assert_same(phi, n, st, gen, p, m, st_ref, g)
