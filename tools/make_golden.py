"""Capture golden vectors from the reference itself (container-only; see tools/refshim.py).

Run from the repo root:  python -m tools.make_golden
Writes tests/golden/*.npz.  Each fixture holds ONLY data: seeds / raw PCG64 states, inputs and the
reference's outputs (fields, acceptance counters, final bit-generator state).  The reference never
travels to the GPU box; these fixtures are the only form in which its behaviour does.

Sources exercised (all /root/reference paths):
  NeighborhoodUpdate.step   supervillain/generator/villain/neighborhood.py:59-137
  SiteUpdate.step           supervillain/generator/villain/site.py:43-118
  LinkUpdate.step           supervillain/generator/villain/link.py:53-99
  ExactUpdate.step          supervillain/generator/villain/exact.py:50-129
  CohomologyUpdate.step     supervillain/generator/villain/cohomology.py:64-117
  CoexactUpdate.step        supervillain/generator/worldline/coexact.py:53-128
  PlaquetteUpdate.step      supervillain/generator/worldline/plaquette.py:35-104
  Lattice.checkerboarding   supervillain/lattice/compact.py:191-239
  Villain/Worldline.__call__ supervillain/action/villain.py:51-66, worldline.py:72-94
  Ensemble.generate         supervillain/ensemble.py:47-100
  Sequentially / KeepEvery  supervillain/generator/combining.py:9-116
"""
import os

import numpy as np

from tools import refshim

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')
MULT = 0x2360ED051FC65DA44385DF649FCCF645
MINV = pow(MULT, -1, 1 << 128)
M128 = (1 << 128) - 1


def rng_state(gen):
    st = gen.bit_generator.state
    return np.array([st['state']['state'] >> 64, st['state']['state'] & ((1 << 64) - 1),
                     st['state']['inc'] >> 64, st['state']['inc'] & ((1 << 64) - 1),
                     st['has_uint32'], st['uinteger']], dtype=np.uint64)


def crafted_generator(seed, position, half):
    """A PCG64 Generator whose raw output number `position` (0-based) has its low (half=0) or
    high (half=1) 32 bits equal to zero, so NumPy's buffered Lemire sampler for k=3 REJECTS the
    uint32 drawn from it.  Natural rejections have probability 2^-32 per draw; this places one
    where a test wants it.  The increment is the one default_rng(seed) picks."""
    gen = np.random.default_rng(seed)
    inc = gen.bit_generator.state['state']['inc']
    hi = 0x0123456789ABCDEF ^ (seed * 0x9E3779B1)  # top 6 bits zero -> rotation 0
    hi &= (1 << 58) - 1
    out = 0xDEADBEEF00000000 if half == 0 else 0x00000000DEADBEEF
    lo = hi ^ out
    s = (hi << 64) | lo
    for _ in range(position + 1):  # undo position+1 steps: s_prev = (s - inc) * M^-1
        s = ((s - inc) * MINV) & M128
    st = gen.bit_generator.state
    st['state']['state'] = s
    st['has_uint32'] = 0
    st['uinteger'] = 0
    gen.bit_generator.state = st
    check = np.random.Generator(np.random.PCG64())
    check.bit_generator.state = st
    raw = check.bit_generator.random_raw(position + 1)[-1]
    assert (int(raw) >> (32 * half)) & 0xFFFFFFFF == 0
    return gen


def villain_chain(sv, N, kappa, W, sweeps, gen, hot_seed=None, interval_phi=np.pi, interval_n=1):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Villain(L, kappa, W)
    G = sv.generator.villain.NeighborhoodUpdate(S, interval_phi=interval_phi, interval_n=interval_n)
    G.rng = gen
    cfg = S.configurations(1)[0]
    if hot_seed is not None:
        r = np.random.default_rng(hot_seed)
        cfg = {'phi': sv.lattice.Form(r.uniform(-np.pi, np.pi, (1, N, N)), degree=0, lattice=L),
               'n': sv.lattice.Form(W * r.integers(-2, 3, (2, N, N)), degree=1, lattice=L)}
    phi0, n0 = np.asarray(cfg['phi'])[0].copy(), np.asarray(cfg['n']).copy()
    rng0 = rng_state(G.rng)
    accepted, acceptance = [], []
    for _ in range(sweeps):
        cfg = G.step(cfg)
        accepted.append(G.accepted)
        acceptance.append(G.acceptance)
    return dict(N=N, kappa=kappa, W=W, sweeps=sweeps, interval_phi=interval_phi, interval_n=interval_n,
                phi0=phi0, n0=n0, rng0=rng0, phi=np.asarray(cfg['phi'])[0].copy(), n=np.asarray(cfg['n']).copy(),
                accepted=np.array(accepted), acceptance=np.array(acceptance), rng1=rng_state(G.rng),
                action=float(S(cfg['phi'], cfg['n'])))


def villain_generator_chain(sv, kind, kw, N, kappa, W, sweeps, gen, hot_seed=None):
    """A chain of one of the SURVEY.md 8(f) Villain generators (Site, Link, Exact, Cohomology)."""
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Villain(L, kappa, W)
    G = getattr(sv.generator.villain, kind)(S, **kw)
    G.rng = gen
    cfg = S.configurations(1)[0]
    if hot_seed is not None:
        r = np.random.default_rng(hot_seed)
        cfg = {'phi': sv.lattice.Form(r.uniform(-np.pi, np.pi, (1, N, N)), degree=0, lattice=L),
               'n': sv.lattice.Form(W * r.integers(-2, 3, (2, N, N)), degree=1, lattice=L)}
    phi0, n0 = np.asarray(cfg['phi'])[0].copy(), np.asarray(cfg['n']).copy()
    rng0 = rng_state(G.rng)
    accepted, acceptance = [], []
    for _ in range(sweeps):
        cfg = G.step(cfg)
        accepted.append(G.accepted)
        acceptance.append(G.acceptance)
    return dict(kind=kind, kw_interval=int(list(kw.values())[0]) if kw else -1, N=N, kappa=kappa, W=W,
                sweeps=sweeps, phi0=phi0, n0=n0, rng0=rng0, phi=np.asarray(cfg['phi'])[0].copy(),
                n=np.asarray(cfg['n']).copy(), accepted=np.array(accepted), acceptance=np.array(acceptance),
                rng1=rng_state(G.rng), report=np.array(G.report()))


def coexact_chain(sv, N, kappa, W, sweeps, seed, vseed, interval_t=1):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Worldline(L, kappa, W)
    G = sv.generator.worldline.CoexactUpdate(S, interval_t=interval_t)
    G.rng = np.random.default_rng(seed)
    r = np.random.default_rng(vseed)
    vdt = int if W < float('inf') else float
    v = (r.integers(-3, 4, (1, N, N)) if vdt is int else r.standard_normal((1, N, N))).astype(vdt)
    cfg = {'m': sv.lattice.Form(np.zeros((2, N, N), dtype=int), degree=1, lattice=L),
           'v': sv.lattice.Form(v, degree=2, lattice=L)}
    rng0 = rng_state(G.rng)
    accepted, acceptance = [], []
    for _ in range(sweeps):
        cfg = cfg | G.step(cfg)
        accepted.append(G.accepted)
        acceptance.append(G.acceptance)
    return dict(N=N, kappa=kappa, W=W, W_eff=S._W, sweeps=sweeps, interval_t=interval_t, v=v[0].copy(), rng0=rng0,
                m=np.asarray(cfg['m']).copy(), accepted=np.array(accepted), acceptance=np.array(acceptance),
                rng1=rng_state(G.rng), action=float(S(cfg['m'], cfg['v'])))


def plaquette_chain(sv, N, kappa, W, sweeps, seed, np_seed):
    L = sv.lattice.Lattice2D(N)
    S = sv.action.Worldline(L, kappa, W)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(seed)
    cfg = S.configurations(1)[0]
    rng0 = rng_state(G.rng)
    saved = np.random.get_state()
    np.random.seed(np_seed)
    orders, accepted, acceptance = [], [], []
    for _ in range(sweeps):
        st = np.random.get_state()
        order = np.random.permutation(L.coordinates)      # what step() is about to draw
        np.random.set_state(st)
        cfg = cfg | G.step(cfg)
        orders.append((order[:, 0] % N) * N + (order[:, 1] % N))
        accepted.append(G.accepted)
        acceptance.append(G.acceptance)
    np.random.set_state(saved)
    return dict(N=N, kappa=kappa, W=W, W_eff=S._W, sweeps=sweeps, np_seed=np_seed, rng0=rng0,
                order=np.array(orders, dtype=np.int64), m=np.asarray(cfg['m']).copy(),
                v=np.asarray(cfg['v'])[0].copy(), accepted=np.array(accepted), acceptance=np.array(acceptance),
                rng1=rng_state(G.rng))


def save(name, cases):
    flat = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            flat[f'{i}/{k}'] = np.asarray(v)
    flat['count'] = np.array(len(cases))
    np.savez_compressed(os.path.join(OUT, name), **flat)
    print(name, len(cases), 'cases')


def main():
    sv = refshim.load()
    os.makedirs(OUT, exist_ok=True)

    # --- NumPy draw KATs (third-party semantics the oracle restates)
    kat = []
    for seed in (0, 1, 12345):
        g = np.random.default_rng(seed)
        c = dict(seed=seed, rng0=rng_state(g))
        c['raw'] = g.bit_generator.random_raw(16)
        c['uniform01'] = g.uniform(0, 1, 33)
        c['uniform_pi'] = g.uniform(-np.pi, np.pi, 33)
        c['choice3'] = g.choice(np.arange(-1, 2), 37)        # odd count leaves a buffered half-word
        c['uniform_after'] = g.uniform(0, 1, 5)             # uniform does not consume the buffer
        c['choice2'] = g.choice((-1, 1), 9)
        c['choice5'] = g.choice(np.arange(-2, 3), 11)
        c['rng1'] = rng_state(g)
        kat.append(c)
    for half in (0, 1):                                   # forced Lemire rejection
        g = crafted_generator(7 + half, 5, half)
        c = dict(seed=-1, rng0=rng_state(g))
        c['raw'] = np.zeros(0, dtype=np.uint64)
        c['uniform01'] = g.uniform(0, 1, 3)
        c['uniform_pi'] = np.zeros(0)
        c['choice3'] = g.choice(np.arange(-1, 2), 8)
        c['uniform_after'] = g.uniform(0, 1, 2)
        c['choice2'] = g.choice((-1, 1), 3)
        c['choice5'] = g.choice(np.arange(-2, 3), 3)
        c['rng1'] = rng_state(g)
        kat.append(c)
    save('rng_kat.npz', kat)

    # --- colourings
    cols = []
    for N in range(2, 12):
        L = sv.lattice.Lattice2D(N)
        cid = np.full((N, N), -1, dtype=np.int32)
        for i, color in enumerate(L.checkerboarding):
            cid[color] = i
        cols.append(dict(N=N, colors=cid))
    save('checkerboarding.npz', cols)

    # --- NeighborhoodUpdate chains
    vil = []
    for N, kappa, W, sweeps, seed, hot in [
            (4, 0.5, 1, 20, 1, None), (4, 0.1, 2, 20, 2, 21),
            (5, 0.5, 1, 30, 3, None), (5, 0.1, 1, 30, 4, 41), (7, 0.3, 2, 25, 5, 51), (9, 0.2, 1, 10, 6, 61),
            (6, 0.1, 1, 20, 7, 71),
            (8, 0.5, 1, 40, 8, None), (8, 0.1, 2, 40, 9, 91), (16, 0.2, 1, 30, 10, 101),
            (16, 0.05, 3, 20, 11, 111), (32, 0.3, 1, 10, 12, 121), (64, 0.2, 2, 5, 13, 131),
            (10, 0.1, 1, 15, 14, 141), (12, 0.15, 1, 15, 15, 151)]:
        vil.append(villain_chain(sv, N, kappa, W, sweeps, np.random.default_rng(seed), hot))
    vil.append(villain_chain(sv, 8, 0.1, 1, 10, np.random.default_rng(16), 161, interval_phi=0.5, interval_n=2))
    vil.append(villain_chain(sv, 8, 0.1, 1, 10, np.random.default_rng(17), 171, interval_n=0))
    save('villain_neighborhood.npz', vil)

    # --- NeighborhoodUpdate with FORCED Lemire rejections (positions in the raw u64 stream)
    rej = []
    V = 64  # N=8: [64 metropolis][colour 0: 32 dphi, 16, 16, 16, 16][colour 1: ...]
    for pos, half, hot in [(64 + 32 + 3, 0, 181), (64 + 32 + 5, 1, 182), (64 + 32 + 16 + 15, 1, 183),
                           (4 * V - 1, 1, 184), (4 * V - 1, 0, 185), (4 * V + 64 + 32 + 2, 0, 186)]:
        rej.append(villain_chain(sv, 8, 0.1, 1, 3, crafted_generator(pos, pos, half), hot))
    # odd N: N=5 colours 7,6,6,6 -> blocks of odd length carry the half-word buffer
    for pos, half, hot in [(25 + 7 + 3, 0, 191), (25 + 7 + 4 + 4 + 4 + 4 + 6 + 2, 1, 192)]:
        rej.append(villain_chain(sv, 5, 0.1, 1, 3, crafted_generator(pos, pos, half), hot))
    save('villain_rejections.npz', rej)

    # --- SiteUpdate, LinkUpdate, ExactUpdate, CohomologyUpdate chains
    more = []
    seed = 300
    for kind, kws in [('SiteUpdate', [{}, {'interval_phi': 0.7}]), ('LinkUpdate', [{}, {'interval_n': 3}]),
                      ('ExactUpdate', [{}, {'interval_z': 2}]), ('CohomologyUpdate', [{}, {'interval_h': 2}])]:
        for kw in kws:
            for N, kappa, W, sweeps, hot in [(4, 0.5, 1, 12, None), (5, 0.3, 1, 10, 1), (8, 0.2, 2, 10, 2),
                                             (16, 0.4, 1, 6, 3), (9, 0.15, 1, 6, 4)]:
                seed += 1
                more.append(villain_generator_chain(sv, kind, kw, N, kappa, W, sweeps, np.random.default_rng(seed),
                                                    None if hot is None else seed * 7 + hot))
    # forced Lemire rejections in LinkUpdate (interval_n=3: 6 choices, threshold 4) and ExactUpdate
    for kind, kw, pos in [('LinkUpdate', {'interval_n': 3}, 5), ('LinkUpdate', {'interval_n': 3}, 40),
                          ('ExactUpdate', {'interval_z': 3}, 64 + 9)]:
        for half in (0, 1):
            more.append(villain_generator_chain(sv, kind, kw, 8, 0.3, 1, 3, crafted_generator(pos, pos, half),
                                                pos * 3 + half))
    save('villain_generators.npz', more)

    # --- CoexactUpdate chains
    co = []
    for N, kappa, W, sweeps, seed in [(4, 0.5, 1, 10, 1), (5, 0.5, 3, 10, 2), (5, 0.4, float('inf'), 10, 3),
                                      (8, 0.5, 1, 20, 4), (8, 0.3, 3, 20, 5), (8, 0.6, float('inf'), 20, 6),
                                      (16, 0.5, 1, 10, 7), (7, 0.5, 2, 10, 8), (32, 0.5, 1, 5, 9),
                                      (6, 0.5, 1, 10, 10)]:
        co.append(coexact_chain(sv, N, kappa, W, sweeps, seed, seed + 100))
    co.append(coexact_chain(sv, 8, 0.5, 1, 10, 11, 111, interval_t=2))
    save('worldline_coexact.npz', co)

    # --- PlaquetteUpdate chains (reference sequential order; permutation recorded)
    pl = []
    for N, kappa, W, sweeps, seed in [(4, 0.5, 1, 5, 1), (5, 0.5, 2, 5, 2), (6, 0.4, float('inf'), 5, 3),
                                      (8, 0.5, 1, 8, 4), (8, 0.3, 3, 5, 5), (16, 0.5, 1, 3, 6)]:
        pl.append(plaquette_chain(sv, N, kappa, W, sweeps, seed, 1000 + seed))
    save('worldline_plaquette.npz', pl)

    # --- Ensemble.generate + composition (host-side boundary behaviour)
    ens = []
    L = sv.lattice.Lattice2D(6)
    S = sv.action.Villain(L, 0.3, 1)
    G = sv.generator.villain.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(5)
    E = sv.Ensemble(S).generate(7, G, starting_index=3, index_stride=2)
    ens.append(dict(kind='villain_generate', N=6, kappa=0.3, W=1, seed=5, steps=7, starting_index=3,
                    index_stride=2, phi=np.asarray(E.configuration.phi.array), n=np.asarray(E.configuration.n.array),
                    index=np.asarray(E.index.array), weight=np.asarray(E.weight.array),
                    report=np.array(G.report())))
    S = sv.action.Worldline(L, 0.5, 1)
    G = sv.generator.worldline.CoexactUpdate(S)
    G.rng = np.random.default_rng(6)
    E = sv.Ensemble(S).generate(5, G)
    ens.append(dict(kind='coexact_generate', N=6, kappa=0.5, W=1, seed=6, steps=5, starting_index=0,
                    index_stride=1, m=np.asarray(E.configuration.m.array), v=np.asarray(E.configuration.v.array),
                    index=np.asarray(E.index.array), weight=np.asarray(E.weight.array), report=np.array(G.report())))
    # Sequentially(NeighborhoodUpdate, NeighborhoodUpdate) inside KeepEvery(3)
    S = sv.action.Villain(L, 0.2, 2)
    a = sv.generator.villain.NeighborhoodUpdate(S)
    b = sv.generator.villain.NeighborhoodUpdate(S, interval_phi=1.0)
    a.rng, b.rng = np.random.default_rng(8), np.random.default_rng(9)
    G = sv.generator.combining.KeepEvery(3, sv.generator.combining.Sequentially((a, b)))
    E = sv.Ensemble(S).generate(4, G)
    ens.append(dict(kind='keepevery_sequentially', N=6, kappa=0.2, W=2, seed=8, steps=4, starting_index=0,
                    index_stride=1, phi=np.asarray(E.configuration.phi.array), n=np.asarray(E.configuration.n.array),
                    index=np.asarray(E.index.array), weight=np.asarray(E.weight.array), report=np.array(G.report())))
    save('ensemble.npz', ens)


if __name__ == '__main__':
    main()
