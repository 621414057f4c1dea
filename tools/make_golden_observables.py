"""Capture the reference's own inline-observable values along seeded Villain chains (container-only; see
tools/refshim.py).  Run from the repo root:  python -m tools.make_golden_observables

Writes tests/golden/villain_observables.npz: per chain the inputs (N, kappa, W, seed, hot-start seed), the
bit-generator states before and after, and after EVERY sweep of NeighborhoodUpdate.step the four scalars the
reference measures on a Villain configuration:

  ActionDensity.Villain          supervillain/observable/action.py:25-31    S(phi, n) / |sites|
  InternalEnergyDensity.Villain  supervillain/observable/energy.py:25-30    S(phi, n) / (|sites| kappa)
  WindingSquared.Villain         supervillain/observable/winding.py:30-37   mean(d(n)**2)
  TorusWrapping.Villain          supervillain/observable/wrapping.py:17-25  n.sum over sites, per direction

computed by those static methods themselves on the reference's own chain (neighborhood.py:59-137).  Chains of one
(N, kappa, W) share a group so that a replica batch (one kappa and W per batch) can run them together.
"""
import os

import numpy as np

from tools import refshim
from tools.make_golden import OUT, rng_state, save

# (group, N, kappa, W, sweeps, seed, hot_seed or None)
CHAINS = [
    ('n8w1', 8, 0.5, 1, 6, 21, None), ('n8w1', 8, 0.5, 1, 6, 22, 221),
    ('n8w2', 8, 0.3, 2, 6, 23, 231), ('n8w2', 8, 0.3, 2, 6, 24, 241),
    ('n16w1', 16, 0.4, 1, 5, 25, 251), ('n16w1', 16, 0.4, 1, 5, 26, 261), ('n16w1', 16, 0.4, 1, 5, 27, None),
    ('n16w2', 16, 0.5, 2, 5, 28, 281), ('n16w2', 16, 0.5, 2, 5, 29, 291),
    ('n128w2', 128, 0.5, 2, 4, 30, 301), ('n128w2', 128, 0.5, 2, 4, 31, 311), ('n128w2', 128, 0.5, 2, 4, 32, None),
    ('n128w1', 128, 0.5, 1, 4, 33, 331), ('n128w1', 128, 0.5, 1, 4, 34, 341),
]


def hot_start(N, W, hot_seed):
    """The hot start of tools/make_golden.villain_chain (phi uniform in [-pi, pi), n in W * {-2..2})."""
    if hot_seed is None:
        return np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    r = np.random.default_rng(hot_seed)
    return r.uniform(-np.pi, np.pi, (1, N, N))[0], (W * r.integers(-2, 3, (2, N, N))).astype(np.int64)


def chain(sv, group, N, kappa, W, sweeps, seed, hot_seed):
    from supervillain.observable.action import ActionDensity
    from supervillain.observable.energy import InternalEnergyDensity
    from supervillain.observable.winding import WindingSquared
    from supervillain.observable.wrapping import TorusWrapping
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Villain(L, kappa, W)
    G = sv.generator.villain.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(seed)
    phi0, n0 = hot_start(N, W, hot_seed)
    cfg = {'phi': sv.lattice.Form(phi0[None].copy(), degree=0, lattice=L),
           'n': sv.lattice.Form(n0.copy(), degree=1, lattice=L)}
    rng0 = rng_state(G.rng)
    ad, ie, w2, tw = [], [], [], []
    for _ in range(sweeps):
        cfg = G.step(cfg)
        phi, n = cfg['phi'], cfg['n']
        ad.append(float(ActionDensity.Villain(S, phi, n)))
        ie.append(float(InternalEnergyDensity.Villain(S, phi, n)))
        w2.append(float(WindingSquared.Villain(S, n)))
        tw.append(np.asarray(TorusWrapping.Villain(S, phi, n), dtype=np.int64))
    return dict(group=group, N=N, kappa=kappa, W=W, sweeps=sweeps, seed=seed,
                hot_seed=-1 if hot_seed is None else hot_seed, rng0=rng0, rng1=rng_state(G.rng),
                ActionDensity=np.array(ad), InternalEnergyDensity=np.array(ie), WindingSquared=np.array(w2),
                TorusWrapping=np.array(tw, dtype=np.int64))


def main():
    sv = refshim.load()
    os.makedirs(OUT, exist_ok=True)
    save('villain_observables.npz', [chain(sv, *c) for c in CHAINS])


if __name__ == '__main__':
    main()
