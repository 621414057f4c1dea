"""Replay the golden reference-order plaquette cases, then the N=32 W=1 oracle case (GPU debug)."""
import sys
import numpy as np
sys.path.insert(0, '.')
import supervillain_amd as sv
from oracle import oracle as O
from tests.golden import cases, generator_from


def golden():
    for c in cases('worldline_plaquette.npz'):
        N = c['N']
        L = sv.Lattice2D(N)
        S = sv.Worldline(L, c['kappa'], c['W'])
        G = sv.generator.worldline.PlaquetteUpdate(S)
        G.rng = generator_from(c['rng0'])
        cfg = S.configurations(1)[0]
        np.random.seed(c['np_seed'])
        for k in range(c['sweeps']):
            cfg = cfg | G.step(cfg)
        print('golden', N, (np.asarray(cfg['m']) == c['m']).all())


def case(N=32, W=1):
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.4, W)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(5)
    cfg = S.configurations(1)[0]
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.int64)
    g = np.random.default_rng(5)
    np.random.seed(77)
    for sweep in range(3):
        st = np.random.get_state()
        o = np.random.permutation(L.coordinates)
        np.random.set_state(st)
        m_before, v_before = np.asarray(cfg['m']).copy(), np.asarray(cfg['v'])[0].copy()
        cfg = cfg | G.step(cfg)
        lin = (o[:, 0] % N) * N + (o[:, 1] % N)
        s = O.worldline_plaquette_seq(N, 0.4, S._W, m, v, lin, g)
        dv = np.argwhere(np.asarray(cfg['v'])[0] != v)
        print('sweep', sweep, 'm diffs', int((np.asarray(cfg['m']) != m).sum()), 'v diffs', len(dv))
        pos = {int(x): i for i, x in enumerate(lin)}
        for t, x in dv:
            print('   site', (t, x), 'visit pos', pos[t * N + x], 'gpu v', np.asarray(cfg['v'])[0][t, x], 'oracle v', v[t, x])
            # neighbours' visit positions
            for dt, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                y = ((t + dt) % N) * N + (x + dx) % N
                print('      nb', ((t + dt) % N, (x + dx) % N), 'pos', pos[y])
        if len(dv):
            break


if __name__ == '__main__':
    golden()
    case()
    case()
