"""Locate a split-replay mismatch: one forced rejection (sweep s, colour c, block j, row, column) at several N,
one sweep per launch (mode 3), against the oracle; prints the mismatching rows / columns."""
import sys
import numpy as np
sys.path.insert(0, '.')
import supervillain_amd as sv  # noqa: E402
from tests.golden import crafted_generator  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(N, sweeps, gen, phi0, n0):
    L = sv.Lattice2D(N)
    S = sv.Villain(L, 0.5, 1)
    G = sv.generator.villain.NeighborhoodUpdate(S, path=2)
    G.rng = gen
    cfg = {'phi': sv.Form(phi0.reshape(1, N, N).copy(), degree=0, lattice=L),
           'n': sv.Form(n0.copy(), degree=1, lattice=L)}
    ctx = G._state()[0]
    ctx.set_multisweep(3, 0)
    ctx.split_counts()
    cfg = G._steps(cfg, sweeps)
    ns = ctx.split_counts()
    c = ctx.sweep_counts()
    ctx.set_multisweep(0, 0)
    return np.asarray(cfg['phi'])[0], np.asarray(cfg['n']), ns, c


for N, sweep, c, j, row, col, sweeps in [(2048, 4, 1, 3, 300, 517, 5), (2048, 0, 1, 3, 300, 517, 1), (1024, 0, 1, 3, 300, 517, 1),
                                          (2048, 0, 1, 3, 100, 517, 1), (2048, 0, 1, 2, 300, 517, 1), (2048, 0, 0, 3, 300, 517, 1),
                                          (4096, 0, 1, 3, 300, 517, 1)]:
    V = N * N
    rank = (row * N + col) // 2
    pos, half = sweep * 4 * V + V + c * (V // 2 + V) + V // 2 + j * (V // 4) + rank // 2, rank % 2
    seed = 300 + 7 * sweep + row
    r = np.random.default_rng(seed)
    phi0, n0 = r.uniform(-np.pi, np.pi, (N, N)), r.integers(-2, 3, (2, N, N)).astype(np.int64)
    p, m = phi0.copy(), n0.copy()
    st = O.villain_neighborhood(N, 0.5, 1, p, m, sweeps, crafted_generator(seed, pos, half))
    phi, n, ns, cnt = run(N, sweeps, crafted_generator(seed, pos, half), phi0, n0)
    bad = np.argwhere(phi != p)
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    print(f'N={N} sweep {sweep} c={c} j={j} row {row} col {col}: rejections {sum(s.rejections for s in st)}, split {ns}, '
          f'{cnt}, phi mismatches {len(bad)}, n mismatches {int((n != m).sum())}; rows {rows[:3]}..{rows[-3:] if rows else []} '
          f'({len(rows)}), cols {cols[:3]}..{cols[-3:] if cols else []} ({len(cols)})', flush=True)
