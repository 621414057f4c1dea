"""Cost of a NumPy Lemire rejection in the driver's window: many back-to-back calls of `steps` L=4096 sweeps
(sv_villain_run path 2, seed-0 chain), each timed on the host; calls that met a rejection vs calls that did not."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 200
Lib = _native.lib()
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
r = rng_from_numpy(np.random.default_rng(0))
st = _native.stats_array(max(steps, 64))


def run(k):
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(r), st, 2), 'run')
    return sum(st[i].rejections for i in range(k))


run(25)
clean, hit = [], []
Lib.sv_ctx_set_timing(ctx.handle, 1)
for c in range(calls):
    t0 = time.perf_counter()
    rj = run(steps)
    dt = time.perf_counter() - t0
    (hit if rj else clean).append(dt)
ms = ctypes.c_double()
nl = ctypes.c_int64()
Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(nl))
counts = ctx.sweep_counts()
c = np.array(clean) * 1e3
hh = np.array(hit) * 1e3
print(f'L={L} steps={steps} calls={calls}: clean {len(c)} calls, median {np.median(c):.3f} ms, mean {c.mean():.3f}; '
      f'with rejection {len(hh)} calls, median {np.median(hh) if len(hh) else 0:.3f} ms, mean {hh.mean() if len(hh) else 0:.3f}; '
      f'extra per rejection call {(np.mean(hh) - np.mean(c)) if len(hh) else 0:.3f} ms; hot kernel {ms.value / max(nl.value, 1) * 1e3:.1f} us '
      f'over {nl.value} launches; sweeps by kernel {counts}', flush=True)
Lib.sv_villain_destroy(h)
