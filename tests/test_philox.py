"""The optional counter-based RNG mode (sv_rng mode 1, "Philox fast") on the CPU oracle: the
generator against the published Philox4x32-10 known-answer vectors (Salmon et al., SC'11; Random123's
kat_vectors), and the Philox NeighborhoodUpdate chain against the reference's own (NumPy PCG64) chain in
distribution -- it is a different Markov chain, so it is tied to the reference statistically, the way
tests/statparity.py ties the checkerboard PlaquetteUpdate.  tests/test_gpu_philox.py pins the device to this
oracle bit for bit."""
import numpy as np


KAT = [  # (counter, key, output)
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers(oracle_lib):
    for ctr, key, out in KAT:
        assert tuple(int(x) for x in oracle_lib.philox4x32_10(ctr, key)) == out


def villain_observables(phi, n, kappa):
    """ActionDensity.Villain (observable/action.py:25-31), the per-direction mean squared residual
    (dphi - 2 pi n)_mu^2 and WindingSquared (observable/winding.py:30-37): functions of the gauge-invariant
    residual, stationary although phi and n themselves random-walk."""
    l0 = (np.roll(phi, -1, axis=0) - phi) - 2 * np.pi * n[0]
    l1 = (np.roll(phi, -1, axis=1) - phi) - 2 * np.pi * n[1]
    dn = (np.roll(n[1], -1, axis=0) - n[1]) - (np.roll(n[0], -1, axis=1) - n[0])
    V = phi.size
    return np.array([kappa / 2 * ((l0 ** 2).sum() + (l1 ** 2).sum()) / V, (l0 ** 2).mean(), (l1 ** 2).mean(),
                     (dn ** 2).mean()])


def _chain(O, mode, N, kappa, W, steps, seed):
    phi = np.zeros((N, N))
    n = np.zeros((2, N, N), dtype=np.int64)
    g = np.random.default_rng(seed)
    out = np.empty((steps, 4))
    for s in range(steps):
        if mode == 'philox':
            O.villain_neighborhood_philox(N, kappa, W, phi, n, 1, 0x5eed0000 + seed, s)
        else:
            O.villain_neighborhood(N, kappa, W, phi, n, 1, g)
        out[s] = villain_observables(phi, n, kappa)
    return out


def test_philox_chain_matches_the_reference_distribution(oracle_lib):
    """Independent chains per mode (the action density decorrelates slowly at N=8, kappa=0.5, so the error comes
    from the chain-to-chain spread, not from blocks of one chain): the per-chain means agree within 4 standard
    errors for every observable."""
    N, kappa, W, steps, cut, chains = 8, 0.5, 1, 12000, 2000, 6
    means = {m: np.array([_chain(oracle_lib, m, N, kappa, W, steps, 10 + c)[cut:].mean(axis=0) for c in range(chains)])
             for m in ('philox', 'pcg64')}
    a, b = means['philox'], means['pcg64']
    se = np.hypot(a.std(axis=0, ddof=1), b.std(axis=0, ddof=1)) / np.sqrt(chains)
    z = (a.mean(axis=0) - b.mean(axis=0)) / se
    assert (np.abs(z) < 4).all(), (z, a.mean(axis=0), b.mean(axis=0), se)


def test_philox_redraws_in_place(oracle_lib):
    """A forced threshold makes about half the choice words redraw; the chain stays a valid Villain chain (n a
    multiple of W) and the redraw count is reported per sweep."""
    N, W = 8, 2
    phi = np.zeros((N, N))
    n = np.zeros((2, N, N), dtype=np.int64)
    st = oracle_lib.villain_neighborhood_philox(N, 0.5, W, phi, n, 4, 77, 0, thr_override=1 << 31)
    assert all(s.rejections > 100 for s in st)
    assert (n % W == 0).all()
