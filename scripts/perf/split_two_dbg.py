"""Debug: two crafted NumPy Lemire rejections in one L=1024 sweep (tests/test_gpu_split.py two-rejection cases) -- where
the device chain departs from the oracle's after one sweep: the differing sites' rows and columns, the kernels that ran."""
import sys

import numpy as np

sys.path.insert(0, '.')
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_split import N, crafted_two, hot, run, word_of  # noqa: E402

CASES = {'same row': ((0, 0, (517 * N + 300) // 2), (0, 2, (517 * N + 600) // 2)),
         'different rows': ((0, 1, (100 * N + 40) // 2), (0, 3, (700 * N + 900) // 2)),
         'both colours': ((0, 2, (333 * N + 123) // 2), (1, 1, (801 * N + 77) // 2)),
         'rows, fwd blocks': ((0, 0, (100 * N + 40) // 2), (0, 2, (700 * N + 900) // 2)),
         'rows, one direction': ((0, 0, (100 * N + 40) // 2), (0, 1, (700 * N + 900) // 2)),
         'rows, interior cols': ((0, 1, (100 * N + 400) // 2), (0, 3, (700 * N + 600) // 2))}
only = sys.argv[1:] or list(CASES)
for name, (a, b) in ((k, CASES[k]) for k in only):
    p1, h1 = word_of(N, *a, 0)
    p2, h2 = word_of(N, *b, 0)
    if (p2 - p1) % 2 == 0:
        b = (b[0], b[1], b[2] + 2)
        p2, h2 = word_of(N, *b, 0)
    seed = 71
    phi0, n0 = hot(N, 1, seed)
    G, phi, n, nsplit, counts = run(N, 1, crafted_two(seed, p1, h1, p2, h2), phi0, n0)
    p, m = phi0.copy(), n0.copy()
    st = O.villain_neighborhood(N, 0.5, 1, p, m, 1, crafted_two(seed, p1, h1, p2, h2))
    bad = np.argwhere((phi != p) | (n != m).any(axis=0))
    print(f'expected skip positions: block {2 + 5 * a[0] + a[1]} pos {a[2]}, block {2 + 5 * b[0] + b[1]} pos {b[2]}')
    print(f'{name}: switches at (c{a[0]} j{a[1]} row {2 * a[2] // N} col {2 * a[2] % N}) and (c{b[0]} j{b[1]} row '
          f'{2 * b[2] // N} col {2 * b[2] % N}); oracle rejections {st[0].rejections}; split sweeps {nsplit}, {counts}; '
          f'{len(bad)} differing sites' + (f', rows {bad[:, 0].min()}..{bad[:, 0].max()}, cols {bad[:, 1].min()}..'
                                           f'{bad[:, 1].max()}, first {bad[:4].tolist()}' if len(bad) else ''), flush=True)
