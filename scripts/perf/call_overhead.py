"""Per-call overhead of sv_villain_run (path 2) at L=4096 in the driver's form (one call of 20 sweeps): wall clock of
the call against the hipEvent time of its hot launches; run with SV_DEBUG_TIMING=1 for the plan / launch / wait
split printed by the library."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L, sweeps, calls = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 20, 6)))
Lib = _native.lib()
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
r = rng_from_numpy(np.random.default_rng(0))
st = _native.stats_array(sweeps)
for c in range(calls):
    Lib.sv_ctx_set_timing(ctx.handle, 1)
    t0 = time.perf_counter()
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, sweeps, ctypes.byref(r), st, 2), 'run')
    dt = time.perf_counter() - t0
    ms, nl = ctypes.c_double(), ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(nl))
    Lib.sv_ctx_set_timing(ctx.handle, 0)
    rej = sum(st[i].rejections for i in range(sweeps))
    print(f'call {c}: wall {dt * 1e6:.0f} us, hot launches {nl.value} x {ms.value / max(nl.value, 1) * 1e3:.1f} us = '
          f'{ms.value * 1e3:.0f} us; overhead {dt * 1e6 - ms.value * 1e3:.0f} us; rejections {rej}', flush=True)
Lib.sv_villain_destroy(h)
