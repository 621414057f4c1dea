"""Repeat the reference-order PlaquetteUpdate vs oracle comparison over many seeds (one process)."""
import sys
import numpy as np
sys.path.insert(0, '.')
import supervillain_amd as sv
from oracle import oracle as O

bad = 0
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
    N = [8, 16, 32, 33, 64][trial % 5]
    W = [1, 2, float('inf')][trial % 3]
    L = sv.Lattice2D(N)
    S = sv.Worldline(L, 0.4, W)
    G = sv.generator.worldline.PlaquetteUpdate(S)
    G.rng = np.random.default_rng(trial)
    cfg = S.configurations(1)[0]
    np.random.seed(1000 + trial)
    m = np.zeros((2, N, N), dtype=np.int64)
    v = np.zeros((N, N), dtype=np.float64 if W == float('inf') else np.int64)
    g = np.random.default_rng(trial)
    for sw in range(3):
        st0 = np.random.get_state()
        o = np.random.permutation(L.coordinates)
        np.random.set_state(st0)
        cfg = cfg | G.step(cfg)
        O.worldline_plaquette_seq(N, 0.4, S._W, m, v, (o[:, 0] % N) * N + (o[:, 1] % N), g)
        ok = (np.asarray(cfg['m']) == m).all() and (np.asarray(cfg['v'])[0] == v).all()
        if not ok:
            bad += 1
            print(f'MISMATCH trial {trial} N={N} W={W} sweep {sw}: m diffs {(np.asarray(cfg["m"]) != m).sum()}')
            break
print('mismatches', bad)
