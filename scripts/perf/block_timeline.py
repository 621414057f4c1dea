"""Workgroup timeline of the temporal-blocking launches (villain_sweep_block; variant built with -DSV_BLKTIME=1): for
the last launch of an L x L chain, medians (and maxima) over the workgroups of
  frame  -- entry -> the frame in LDS (small-offset maps, phi / n loads)
  bases  -- -> row bases ready (the table jumps)
  sweep j -- -> sweep j's own block stored
  exit   -- -> statistics added
and the launch's span (latest exit minus earliest entry).  Usage:
  SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_blktime.so python scripts/perf/block_timeline.py [L] [sweeps] [K]"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 63
K = int(sys.argv[3]) if len(sys.argv) > 3 else 3
Lib = _native.lib()
Lib.sv_debug_blocktime.argtypes = [ctypes.c_void_p, ctypes.c_int32]
ctx = _native.context()
ctx.set_multisweep(1, K)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
nwg = 4096
buf = np.zeros(nwg * 16, dtype=np.uint64)
for rep in range(3):
    g = np.random.default_rng(rep)
    r = rng_from_numpy(g)
    st = _native.stats_array(sweeps)
    ctx.block_counts()
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, sweeps, ctypes.byref(r), st, 2), 'run')
    bc = ctx.block_counts()
    buf[:] = 0
    assert Lib.sv_debug_blocktime(buf.ctypes.data, nwg) == 0
    t = buf.reshape(nwg, 16).astype(np.int64)
    m = t[:, 0] > 0
    t = t[m]
    kk = bc['sweeps'] // max(bc['launches'], 1)
    t0 = t[:, 0].min()
    cols = [('frame', 0, 1), ('bases', 1, 2)] + [(f'sweep{j}', 2 + j, 3 + j) for j in range(kk)] + \
        [('exit', 2 + kk, 15)]
    out = []
    for name, a, b in cols:
        d = (t[:, b] - t[:, a]) * 0.01
        out.append(f'{name} {np.median(d):5.2f} (max {d.max():5.2f})')
    ent = (t[:, 0] - t0) * 0.01
    span = (t[:, 15].max() - t0) * 0.01
    print(f'[L={L} rep {rep}] {bc}, WGs {len(t)}, entry spread {ent.max():5.2f} us: ' + '  '.join(out) +
          f'  span {span:6.2f} us')
ctx.check(Lib.sv_villain_destroy(h), 'destroy')
