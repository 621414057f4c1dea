"""Tail-recovery potential: two independent L x L chains on two contexts (streams), driven from two host threads,
against one chain alone.  If the per-sweep throughput of the pair beats the single chain, the single chain's
launch tails (the last, partly filled round of workgroup slots) are what the difference costs."""
import ctypes
import sys
import threading
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
Lib = _native.lib()


class Chain:
    def __init__(self, seed):
        self.ctx = _native.Context(0)
        self.h = ctypes.c_void_p()
        self.ctx.check(Lib.sv_villain_create(self.ctx.handle, L, ctypes.byref(self.h)), 'create')
        phi = np.zeros((L, L))
        n = np.zeros((2, L, L), dtype=np.int64)
        self.ctx.check(Lib.sv_villain_upload(self.h, _native.ptr(phi), _native.ptr(n)), 'upload')
        self.r = rng_from_numpy(np.random.default_rng(seed))
        self.st = _native.stats_array(max(sweeps, 64))

    def run(self, k):
        self.ctx.check(Lib.sv_villain_run(self.h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(self.r), self.st, 2), 'run')


a, b = Chain(0), Chain(1)
a.run(10)
b.run(10)
for rep in range(3):
    t0 = time.perf_counter()
    a.run(sweeps)
    t1 = time.perf_counter()
    ths = [threading.Thread(target=c.run, args=(sweeps,)) for c in (a, b)]
    t2 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t3 = time.perf_counter()
    print(f'L={L}: one chain {(t1 - t0) / sweeps * 1e6:.1f} us per sweep; two concurrent chains '
          f'{(t3 - t2) / (2 * sweeps) * 1e6:.1f} us per sweep each-equivalent', flush=True)
