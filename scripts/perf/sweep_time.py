"""Per-sweep time of sv_villain_run (path 2) at several L: wall clock over `sweeps` sweeps in one call, and the
hipEvent time of the hot launches, the seed-0 cold chain.  Usage: sweep_time.py sweeps L..."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

sweeps = int(sys.argv[1])
Lib = _native.lib()
ctx = _native.context(0)
for L in [int(x) for x in sys.argv[2:]]:
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
    r = rng_from_numpy(np.random.default_rng(0))
    st = _native.stats_array(sweeps)

    def run(k):
        ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(r), st, 2), 'run')
        return sum(st[i].rejections for i in range(k))

    run(20)
    out = []
    for rep in range(3):
        Lib.sv_ctx_set_timing(ctx.handle, 1)
        t0 = time.perf_counter()
        rj = run(sweeps)
        dt = time.perf_counter() - t0
        ms, nl = ctypes.c_double(), ctypes.c_int64()
        Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(nl))
        Lib.sv_ctx_set_timing(ctx.handle, 0)
        out.append((dt / sweeps * 1e6, ms.value / max(nl.value, 1) * 1e3, rj))
    print(f'L={L}: ' + '; '.join(f'wall {w:.1f} us/sweep, events {e:.1f} (rej {j})' for w, e, j in out), flush=True)
    Lib.sv_villain_destroy(h)
