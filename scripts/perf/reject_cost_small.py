"""Cost of one NumPy Lemire rejection on a small lattice (config 2, L=256: temporal-blocking launches): calls of
`steps` sweeps from a crafted PCG64 state that makes one bounded draw of sweep `at` a rejection, against the same
calls from crafted states whose rejection lies beyond the call (clean), timed on the host, interleaved.

    python scripts/perf/reject_cost_small.py [L=256] [steps=200] [reps=30] [at=100]"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402
from tests.golden import crafted_generator  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
at = int(sys.argv[4]) if len(sys.argv) > 4 else 100
V = L * L
Lib = _native.lib()
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
r0 = np.random.default_rng(1)
phi = r0.uniform(-np.pi, np.pi, (L, L))
n = r0.integers(-2, 3, (2, L, L)).astype(np.int64)
st = _native.stats_array(steps)


def call(sweep_of_rejection, seed):
    ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
    pos = sweep_of_rejection * 4 * V + V + V // 2 + 7  # a colour-0 choice block of that sweep
    r = rng_from_numpy(crafted_generator(seed, pos, 0))
    t0 = time.perf_counter()
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, steps, ctypes.byref(r), st, 2), 'run')
    dt = time.perf_counter() - t0
    return dt, sum(st[i].rejections for i in range(steps))


call(at, 5)
call(steps + 10, 5)
hit, clean = [], []
for i in range(reps):
    dt, rj = call(at, 100 + i)
    assert rj == 1, rj
    hit.append(dt)
    dt, rj = call(steps + 10, 100 + i)  # (the crafted word lies after the call: a clean call)
    assert rj == 0, rj
    clean.append(dt)
hit, clean = np.array(hit) * 1e6, np.array(clean) * 1e6
counts = ctx.sweep_counts()
print(f'L={L} {steps} sweeps per call, rejection at sweep {at}: clean median {np.median(clean):.1f} us '
      f'({np.median(clean) / steps:.2f} us per sweep), with the rejection median {np.median(hit):.1f} us; '
      f'cost of the rejection {np.median(hit) - np.median(clean):.1f} us (mean {hit.mean() - clean.mean():.1f}); '
      f'block {ctx.block_counts()}, split {ctx.split_counts()}, sweeps by kernel {counts}', flush=True)
Lib.sv_villain_destroy(h)
