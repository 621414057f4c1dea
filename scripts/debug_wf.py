"""Debug: one fused Worldline step vs the four pass kernels (SV_WF toggled per call)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy

def run(N, wf, steps=1, seed=9):
    os.environ['SV_WF'] = '1' if wf else '0'
    r0 = np.random.default_rng(N + 1)
    v0 = r0.integers(-2, 3, (N, N)).astype(np.int64)
    m0 = np.zeros((2, N, N), dtype=np.int64)
    Lib = _native.lib(); ctx = _native.context(0)
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, N, 0, ctypes.byref(h)), 'create')
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m0), _native.ptr(v0)), 'upload')
    r = rng_from_numpy(np.random.default_rng(seed))
    st = _native.stats_array(2 * steps)
    ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, 0.5, 1.0, 1, steps, ctypes.byref(r), st), 'run')
    m, v = np.empty_like(m0), np.empty_like(v0)
    ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'download')
    Lib.sv_worldline_destroy(h)
    return m, v, [(st[i].accepted, st[i].acceptance_sum) for i in range(2 * steps)]

for N in (8, 16, 64, 128, 256):
    a = run(N, True); b = run(N, False)
    print(N, 'm equal', (a[0] == b[0]).all(), 'v equal', (a[1] == b[1]).all(), 'stats', a[2], b[2], flush=True)
    if not (a[0] == b[0]).all():
        d = np.argwhere(a[0] != b[0]); print('  m diffs', len(d), d[:10].tolist())
    if not (a[1] == b[1]).all():
        d = np.argwhere(a[1] != b[1]); print('  v diffs', len(d), d[:10].tolist())
