"""worldline_step_fused's turned strip layout (16-wave launches on periodic lattices): the column strips turned
left by half a strip so that strip 0 alone holds the torus's column seam, in short row strips, and the row bases
moved across the row seam by the inverse advance maps.  Bit-exact against the oracle at config 3's size with
forced NumPy Lemire rejections (the GENERAL-mode replay in the turned layout), and against the plain layout
(SV_WF_TURN=0) over batch boundaries at both 16-wave sizes and W = 1, 2.

Reference: plaquette.py:84-85 (checkerboard PlaquetteUpdate), coexact.py:96-120 (CoexactUpdate)."""
import numpy as np
import pytest

from tests.golden import crafted_generator
from tests.test_gpu_worldline import _worldline_run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('which', ['step0 colour0 change_v', 'step1 colour1 change_v'])
def test_turned_layout_forced_rejection_at_config3(which, oracle_lib):
    """A rejection forced into a change_v block at L = 1024 (raw u64 positions as in
    test_gpu_worldline.py::test_plaquette_coexact_forced_rejection), replayed in the GENERAL mode of the turned
    layout; three steps against the oracle step by step."""
    N = 1024
    V = N * N
    per_step = 2 * V + V + V // 2
    pos, half = {'step0 colour0 change_v': (V + V // 4 + 3, 0),
                 'step1 colour1 change_v': (per_step + V + 3 * V // 4 + 1, 1)}[which]
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
        np.testing.assert_allclose([st[2 * s].acceptance_sum, st[2 * s + 1].acceptance_sum],
                                   [sp.acceptance_sum, sc.acceptance_sum], rtol=1e-12)
    assert rej >= 1
    assert (m == mm).all() and (v == vv).all()
    assert gen.bit_generator.state == g.bit_generator.state


@pytest.mark.parametrize('N,W', [(1024, 1.0), (960, 2.0), (1024, 0.5)])
def test_turned_layout_equals_plain_layout(N, W, monkeypatch):
    """70 steps (across the 64-step batch) from a random v: the turned layout's fields, accepted counts, acceptance
    sums and NumPy state, with and without the last row strip cut in two (SV_WF_TAIL=0), equal the plain layout's
    (SV_WF_TURN=0; both read per call) bit for bit."""
    v0 = np.random.default_rng(N).integers(-3, 4, (N, N)).astype(np.int64)
    m0 = np.zeros((2, N, N), dtype=np.int64)
    out = {}
    for turn, tail in (('1', '1'), ('1', '0'), ('0', '1')):
        monkeypatch.setenv('SV_WF_TURN', turn)
        monkeypatch.setenv('SV_WF_TAIL', tail)
        gen = np.random.default_rng(9)
        m, v, st = _worldline_run(N, 0.5, W, m0, v0, 70, gen)
        out[turn + tail] = (m, v, [(s.accepted, s.acceptance_sum, s.rejections) for s in st], gen.bit_generator.state)
    for key in ('11', '10'):
        a, b = out[key], out['01']
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all(), key
        assert [x[0] for x in a[2]] == [x[0] for x in b[2]], key
        assert [x[2] for x in a[2]] == [x[2] for x in b[2]], key
        # the float acceptance sums are exact sums (common.h): equal bit for bit whatever the strip layout
        assert [x[1] for x in a[2]] == [x[1] for x in b[2]], key
        assert a[3] == b[3], key
