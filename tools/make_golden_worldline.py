"""Golden vectors for the SURVEY.md 8(f) row-2 Worldline generators, captured from the reference itself
(container-only; tools/refshim.py).  Run from the repo root:  python -m tools.make_golden_worldline
Writes tests/golden/worldline_generators.npz (data only: inputs, outputs, counters, PCG64 states).

Sources exercised (all /root/reference paths):
  VortexUpdate.step    supervillain/generator/worldline/vortex.py:51-136
  WrappingUpdate.step  supervillain/generator/worldline/wrapping.py:43-90
  Hammer (minus worm)  supervillain/generator/worldline/__init__.py:10-40
"""
import numpy as np

from tools import refshim
from tools.make_golden import crafted_generator, rng_state, save


def hot(sv, L, W, N, seed):
    """A hot (m, v): m with dm = 0 is not needed by these generators, but a coexact-built m keeps the
    configuration physical (m = delta(t) for a random integer 2-form t)."""
    r = np.random.default_rng(seed)
    t = sv.lattice.Form(r.integers(-2, 3, (1, N, N)), degree=2, lattice=L)
    m = np.asarray(sv.lattice.delta(t)).astype(int)
    if W < float('inf'):
        v = W * r.integers(-2, 3, (1, N, N))
    else:
        v = r.standard_normal((1, N, N))
    return m, v


def chain(sv, kind, kw, N, kappa, W, sweeps, gen, seed):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Worldline(L, kappa, W)
    G = getattr(sv.generator.worldline, kind)(S, **kw)
    G.rng = gen
    m, v = hot(sv, L, W, N, seed)
    cfg = {'m': sv.lattice.Form(m, degree=1, lattice=L), 'v': sv.lattice.Form(v, degree=2, lattice=L)}
    m0, v0 = np.asarray(cfg['m']).copy(), np.asarray(cfg['v'])[0].copy()
    rng0 = rng_state(G.rng)
    accepted, acceptance = [], []
    for _ in range(sweeps):
        cfg = cfg | G.step(cfg)
        accepted.append(G.accepted)
        acceptance.append(G.acceptance)
    return dict(kind=kind, kw_interval=int(list(kw.values())[0]) if kw else -1, N=N, kappa=kappa, W=W, W_eff=S._W,
                sweeps=sweeps, m0=m0, v0=v0, rng0=rng0, m=np.asarray(cfg['m']).copy(),
                v=np.asarray(cfg['v'])[0].copy(), accepted=np.array(accepted), acceptance=np.array(acceptance),
                rng1=rng_state(G.rng), report=np.array(G.report()))


def main():
    sv = refshim.load()
    out = []
    params = [(4, 0.5, 1, 8, 1), (5, 0.3, 1, 6, 2), (8, 0.2, 2, 6, 3), (6, 0.4, float('inf'), 6, 4),
              (9, 0.6, 3, 4, 5), (16, 0.5, 1, 4, 6), (7, 0.35, float('inf'), 4, 7), (32, 0.25, 2, 3, 8)]
    for kind, kws in [('VortexUpdate', [{}, {'interval_v': 2}]), ('WrappingUpdate', [{}, {'interval_w': 3}])]:
        for kw in kws:
            for N, kappa, W, sweeps, seed in params:
                out.append(chain(sv, kind, kw, N, kappa, W, sweeps, np.random.default_rng(seed + 40), seed + 60))
    # forced NumPy Lemire rejections (k = 6: interval 3) inside the bounded draws
    for kind, kw, pos in [('VortexUpdate', {'interval_v': 3}, 64 + 5), ('WrappingUpdate', {'interval_w': 3}, 3)]:
        for half in (0, 1):
            out.append(chain(sv, kind, kw, 8, 0.3, 1, 2, crafted_generator(pos, pos, half), 90 + half))
    save('worldline_generators.npz', out)


if __name__ == '__main__':
    main()
