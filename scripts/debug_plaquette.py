"""Diagnose reference-order PlaquetteUpdate differences between the device and the oracle."""
import sys
import numpy as np
sys.path.insert(0, '.')
import supervillain_amd as sv
from oracle import oracle as O

N, W, kappa = int(sys.argv[1]), float(sys.argv[2]), 0.4
L = sv.Lattice2D(N)
S = sv.Worldline(L, kappa, W)
G = sv.generator.worldline.PlaquetteUpdate(S)
G.rng = np.random.default_rng(5)
cfg = S.configurations(1)[0]
np.random.seed(77)
m = np.zeros((2, N, N), dtype=np.int64)
v = np.zeros((N, N), dtype=np.float64 if W == float('inf') else np.int64)
g = np.random.default_rng(5)
for sw in range(3):
    st0 = np.random.get_state()
    o = np.random.permutation(L.coordinates)
    np.random.set_state(st0)
    cfg = cfg | G.step(cfg)
    lin = (o[:, 0] % N) * N + (o[:, 1] % N)
    s = O.worldline_plaquette_seq(N, kappa, S._W, m, v, lin, g)
    dm = np.argwhere(np.asarray(cfg['m']) != m)
    dv = np.argwhere(np.asarray(cfg['v'])[0] != v)
    print(f'sweep {sw}: oracle acc {s.accepted} gpu acc total {G.accepted}; m diffs {len(dm)} v diffs {len(dv)}')
    if len(dv):
        pos = {int(x): i for i, x in enumerate(lin)}
        for t, x in dv[:10]:
            print('  v diff at', (t, x), 'visit pos', pos[t * N + x], 'gpu', np.asarray(cfg['v'])[0][t, x], 'oracle', v[t, x])
        break
