"""Statistical parity of the checkerboard PlaquetteUpdate chain against the reference's sequential chain, on the
CPU oracle (tests/statparity.py says why and how).

Both chains here are the oracle's restatements: `worldline_plaquette_seq` is pinned bit for bit to the
reference's PlaquetteUpdate by tests/golden/worldline_plaquette.npz (test_oracle_golden.py), and
`worldline_plaquette_cb` is the checkerboard chain the GPU kernel matches bit for bit
(tests/test_gpu_worldline.py).  So agreement here ties the GPU's checkerboard chain to the reference's
distribution; tests/test_gpu_worldline.py::test_plaquette_checkerboard_statistical_parity repeats the
comparison with both chains on the GPU.
"""
import numpy as np
import pytest

from tests.statparity import NAMES, compare, observables

N, KAPPA, W = 8, 0.5, 1.0
STEPS, CUT = 20000, 1000


def _chain(O, mode, steps, seed):
    """Plaquette (checkerboard or reference order) + Coexact per step from a cold start; observables per step."""
    g = np.random.default_rng(seed)
    legacy = np.random.RandomState(seed + 1)  # the reference's global RandomState permutation (plaquette.py:63)
    coords = np.array([(t, x) for t in range(N) for x in range(N)])
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.int64)
    out = np.empty((steps, len(NAMES)))
    for s in range(steps):
        if mode == 'checkerboard':
            O.worldline_plaquette_cb(N, KAPPA, W, m, v, 1, g)
        else:
            order = legacy.permutation(coords)
            O.worldline_plaquette_seq(N, KAPPA, W, m, v, (order[:, 0] % N) * N + order[:, 1] % N, g)
        O.worldline_coexact(N, KAPPA, W, m, v, 1, g)
        out[s] = observables(m, v, KAPPA, W)
    return out


def test_checkerboard_plaquette_matches_reference_distribution(oracle_lib):
    cb = _chain(oracle_lib, 'checkerboard', STEPS, 1)
    ref = _chain(oracle_lib, 'reference', STEPS, 2)
    zs = compare(cb, ref, CUT)
    for name, (z, ma, ea, mb, eb) in zs.items():
        assert abs(z) < 4.0, f'{name}: checkerboard {ma:.5f} +- {ea:.5f} vs reference order {mb:.5f} +- {eb:.5f}'
    # the errors are meaningful (a frozen chain would pass the z test with zero variance)
    assert all(0 < zs[n][2] < 0.01 for n in NAMES)


def test_statistics_detect_a_wrong_distribution(oracle_lib):
    """The comparison has power: the same chain at a different kappa (a different distribution) fails it."""
    global KAPPA
    ref = _chain(oracle_lib, 'reference', STEPS // 2, 2)
    saved = KAPPA
    try:
        KAPPA = 0.45
        other = _chain(oracle_lib, 'checkerboard', STEPS // 2, 1)
    finally:
        KAPPA = saved
    zs = compare(other, ref, CUT)
    # F2 (mean squared f per direction) does not involve kappa in its definition: a pure distribution change
    assert abs(zs['F2_0'][0]) > 4.0 and abs(zs['F2_1'][0]) > 4.0, zs
