"""Statistical parity of two Markov chains with the same stationary distribution (test helper).

The checkerboard PlaquetteUpdate (`mode='checkerboard'`, the GPU-native chain bench.py's config 3 times) is a
different Markov chain from the reference's sequential permutation sweep
(/root/reference/supervillain/generator/worldline/plaquette.py:35-104), so it cannot be checked bit for bit
against the reference.  It is checked the way the reference compares its own algorithms
(/root/reference/example/worldline-algorithm-comparison.py:38-95): run both chains, cut thermalization,
measure an observable per configuration, estimate each mean with a blocked bootstrap (blocks much longer
than the autocorrelation time) and require agreement within a few standard errors.

Observables (Worldline formulation, D=2):
  ActionDensity.Worldline  (L.links/2 - 0.5/kappa * sum (m - delta v / W)^2) / L.sites
                           /root/reference/supervillain/observable/action.py:37-50
  F2_mu                    mean over sites of (m - delta v / W)_mu^2, per direction mu (the two halves of
                           the action; equal by the lattice's rotation symmetry)
m and v alone random-walk at W=1 (a plaquette move with change_m = change_v leaves f = m - delta v / W
unchanged and is always accepted), so only functions of f are stationary.
"""
import numpy as np


def delta_v(v, W):
    """delta of the 2-form v as a 1-form, D=2 (('delta', 2) rows (0,0,1,-1), (1,0,0,+1)):
    (delta v)_0[x] = v[x] - v[x - e1], (delta v)_1[x] = -v[x] + v[x - e0]."""
    v2 = np.asarray(v, dtype=np.float64).reshape(v.shape[-2:])
    return np.stack([v2 - np.roll(v2, 1, axis=1), -v2 + np.roll(v2, 1, axis=0)]) / W


def observables(m, v, kappa, W):
    N = m.shape[-1]
    f = np.asarray(m, dtype=np.float64) - delta_v(v, W)
    links, sites = 2 * N * N, N * N
    return np.array([(links / 2 - 0.5 / kappa * (f ** 2).sum()) / sites, (f[0] ** 2).mean(), (f[1] ** 2).mean()])


NAMES = ('ActionDensity', 'F2_0', 'F2_1')


def blocked_bootstrap(x, blocks=100, samples=400, seed=0):
    """Mean and standard error of the mean of a correlated series: the series is cut into `blocks` contiguous
    blocks and the block means are bootstrap-resampled."""
    x = np.asarray(x, dtype=np.float64)
    b = x[:len(x) // blocks * blocks].reshape(blocks, -1).mean(axis=1)
    rng = np.random.default_rng(seed)
    boot = b[rng.integers(0, blocks, (samples, blocks))].mean(axis=1)
    return b.mean(), boot.std(ddof=1)


def compare(a, b, cut, blocks=100):
    """z-scores (mean_a - mean_b) / sqrt(err_a^2 + err_b^2) per observable column, after cutting `cut`
    thermalization steps from each series."""
    zs = {}
    for k, name in enumerate(NAMES):
        ma, ea = blocked_bootstrap(a[cut:, k], blocks)
        mb, eb = blocked_bootstrap(b[cut:, k], blocks)
        zs[name] = ((ma - mb) / np.hypot(ea, eb), ma, ea, mb, eb)
    return zs
