"""Golden vectors for SURVEY.md 8(f) row 4 (the worms), captured from the reference itself (container-only;
tools/refshim.py).  Run from the repo root:  python -m tools.make_golden_worm
Writes tests/golden/worms.npz (data only: inputs, per-step outputs, PCG64 states).

Sources exercised (all /root/reference paths):
  villain ClassicWorm.step    supervillain/generator/villain/worm.py:85-131, worm_kernel :133-183
  worldline ClassicWorm.step  supervillain/generator/worldline/worm.py:137-193, worm_kernel :26-94
  _Lattice2D moves            supervillain/lattice/two_dimensional.py:221-300
  Hammer (worm included) through Ensemble.generate: villain/__init__.py:11-67, worldline/__init__.py:10-40,
                              ensemble.py:47-100, combining.py:9-116 (worms.npz 'hammer' cases)
"""
import numpy as np

from tools import refshim
from tools.make_golden import rng_state, save


def villain_case(sv, N, kappa, W, steps, seed, hot):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Villain(L, kappa, W)
    G = sv.generator.villain.Worm(S)
    G.rng = np.random.default_rng(seed)
    r = np.random.default_rng(seed + 1000)
    phi = np.zeros((1, N, N))
    n = np.zeros((2, N, N), dtype=np.int64)
    cfg = {'phi': sv.lattice.Form(phi, degree=0, lattice=L), 'n': sv.lattice.Form(n, degree=1, lattice=L)}
    if hot and W < float('inf'):
        # a thermalized start: 30 reference NeighborhoodUpdate sweeps (hot random n makes worms that never close)
        T = sv.generator.villain.NeighborhoodUpdate(S)
        T.rng = r
        for _ in range(30):
            cfg = cfg | T.step(cfg)
    elif hot:
        cfg['phi'] = sv.lattice.Form(r.uniform(-np.pi, np.pi, (1, N, N)), degree=0, lattice=L)
    phi, n = np.asarray(cfg['phi']).copy(), np.asarray(cfg['n']).copy()
    rng0 = rng_state(G.rng)
    hists, lengths = [], []
    for _ in range(steps):
        cfg = cfg | G.step(cfg)
        hists.append(np.asarray(cfg['Vortex_Vortex']).copy())
        lengths.append(int(cfg['Worm_Length']))
    return dict(action='villain', N=N, kappa=kappa, W=W, steps=steps, phi0=phi[0].copy(), n0=n.copy(), rng0=rng0,
                n=np.asarray(cfg['n']).copy(), hist=np.array(hists), lengths=np.array(lengths),
                rng1=rng_state(G.rng), report=np.array(G.report()))


def worldline_case(sv, N, kappa, W, steps, seed, hot):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Worldline(L, kappa, W)
    G = sv.generator.worldline.Worm(S)
    G.rng = np.random.default_rng(seed)
    r = np.random.default_rng(seed + 2000)
    m = np.zeros((2, N, N), dtype=np.int64)
    if hot:
        v = W * r.integers(-2, 3, (1, N, N)) if W < float('inf') else r.standard_normal((1, N, N))
    else:
        v = np.zeros((1, N, N), dtype=np.int64 if W < float('inf') else np.float64)
    cfg = {'m': sv.lattice.Form(m, degree=1, lattice=L), 'v': sv.lattice.Form(v, degree=2, lattice=L)}
    if hot:  # thermalized m: 30 reference CoexactUpdate sweeps (keeps delta m = 0)
        T = sv.generator.worldline.CoexactUpdate(S)
        T.rng = r
        for _ in range(30):
            cfg = cfg | T.step(cfg)
    m, v = np.asarray(cfg['m']).copy(), np.asarray(cfg['v']).copy()
    rng0 = rng_state(G.rng)
    hists, lengths = [], []
    for _ in range(steps):
        cfg = cfg | G.step(cfg)
        hists.append(np.asarray(cfg['Spin_Spin']).copy())
        lengths.append(int(cfg['Worm_Length']))
    return dict(action='worldline', N=N, kappa=kappa, W=W, W_eff=S._W, steps=steps, m0=m.copy(), v0=v[0].copy(),
                rng0=rng0, m=np.asarray(cfg['m']).copy(), hist=np.array(hists), lengths=np.array(lengths),
                rng1=rng_state(G.rng), report=np.array(G.report()))


def hammer_case(sv, action, N, kappa, W, steps, seed, worms):
    """Ensemble(S).generate(steps, Hammer(S, worms)) from a cold start, every member generator seeded."""
    L = sv.lattice.Lattice2D(N)
    S = (sv.action.Villain if action == 'villain' else sv.action.Worldline)(L, kappa, W)
    H = (sv.generator.villain if action == 'villain' else sv.generator.worldline).Hammer(S, worms)
    seeds = []
    for i, G in enumerate(H.generators):
        g = G.generator if hasattr(G, 'stride') else G
        g.rng = np.random.default_rng(seed + i)
        seeds.append(seed + i)
    E = sv.Ensemble(S).generate(steps, H)
    key = 'Vortex_Vortex' if action == 'villain' else 'Spin_Spin'
    fields = ('phi', 'n') if action == 'villain' else ('m', 'v')
    out = dict(action='hammer_' + action, N=N, kappa=kappa, W=W, steps=steps, worms=worms, seeds=np.array(seeds),
               hist=np.asarray(getattr(E, key)).copy(), lengths=np.asarray(E.Worm_Length).copy(),
               report=np.array(H.report()))
    for f in fields:
        out[f] = np.asarray(getattr(E, f)).copy()
    return out


def main():
    sv = refshim.load()
    out = []
    for N, kappa, W, steps, seed, hot in [(4, 0.5, 1, 12, 1, False), (5, 0.3, 2, 10, 2, True), (8, 0.2, 2, 8, 3, True),
                                          (6, 0.7, 3, 8, 4, True), (7, 0.4, float('inf'), 8, 5, True),
                                          (8, 0.5, 1, 8, 6, True), (16, 0.25, 2, 4, 7, True), (12, 0.6, 1, 4, 8, False),
                                          (8, 1.0, 1, 6, 9, True), (6, 1.2, 2, 6, 10, True)]:
        out.append(villain_case(sv, N, kappa, W, steps, seed, hot))
    for N, kappa, W, steps, seed, hot in [(4, 0.5, 1, 12, 11, False), (5, 0.3, 2, 10, 12, True), (8, 0.2, 1, 8, 13, True),
                                          (6, 0.7, 3, 8, 14, True), (7, 0.4, float('inf'), 8, 15, True),
                                          (16, 0.5, 2, 4, 16, True), (9, 1.0, 1, 6, 17, False)]:
        out.append(worldline_case(sv, N, kappa, W, steps, seed, hot))
    for action, N, kappa, W, steps, seed, worms in [('villain', 8, 0.5, 2, 5, 100, 1), ('villain', 6, 0.7, 1, 4, 110, 1),
                                                      ('villain', 8, 0.6, 3, 3, 115, 3),
                                                      ('worldline', 8, 0.5, 1, 5, 120, 1),
                                                      ('worldline', 6, 0.4, 2, 4, 130, 1),
                                                      ('worldline', 6, 0.6, float('inf'), 3, 140, 2)]:
        out.append(hammer_case(sv, action, N, kappa, W, steps, seed, worms))
    for c in out:
        print(c['action'], c['N'], c['kappa'], c['W'], 'lengths', np.asarray(c['lengths']).tolist())
    save('worms.npz', out)


if __name__ == '__main__':
    main()
