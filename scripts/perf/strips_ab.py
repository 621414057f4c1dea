"""A/B of villain_sweep_hot strip schedules (SV_STRIPS) on one L x L lattice: hipEvent time per hot launch over a few
hundred sweeps, interleaved repetitions.  Usage: python scripts/perf/strips_ab.py L sweeps reps spec1 spec2 ..."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L, sweeps, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
specs = [s if s != 'uniform' else '' for s in sys.argv[4:]]
Lib = _native.lib()
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
r = rng_from_numpy(np.random.default_rng(0))
st = _native.stats_array(sweeps)


def run(k):
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(r), st, 2), 'run')


run(20)
res = {s: [] for s in specs}
for rep in range(reps):
    for s in specs:
        os.environ['SV_STRIPS'] = s
        run(4)
        Lib.sv_ctx_set_timing(ctx.handle, 1)
        run(sweeps)
        ms, nl = ctypes.c_double(), ctypes.c_int64()
        Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(nl))
        Lib.sv_ctx_set_timing(ctx.handle, 0)
        res[s].append(ms.value / max(nl.value, 1) * 1e3)
for s in specs:
    print(f'L={L} strips "{s or "uniform"}": ' + ' '.join(f'{v:.1f}' for v in res[s]) + f' us per hot sweep (mean {np.mean(res[s]):.1f})',
          flush=True)
Lib.sv_villain_destroy(h)
