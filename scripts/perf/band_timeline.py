"""Per-sweep timeline of the multi-sweep band launches (villain_sweep_hot_band; variant built with -DSV_WGTIME=1):
for the last band launch of an L x L chain, per sweep j of the launch, the medians over the busy workgroups of
  start   -- from the previous barrier (or the first entry) to hot_body's entry
  bases   -- entry -> row bases ready (the prologue's table jumps)
  rows    -- bases -> loop start (first row loads, commit, barrier)
  loop    -- the row steps
  epi     -- loop end -> exit (last stores, statistics)
  barrier -- exit -> band barrier passed
and the sweep's span (latest barrier pass minus the earliest barrier pass of the previous sweep).  Usage:
  SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so python scripts/perf/band_timeline.py [L] [sweeps]"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 63
Lib = _native.lib()
Lib.sv_debug_bandtime.argtypes = [ctypes.c_void_p, ctypes.c_int32]
ctx = _native.context()
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
slots = 8 * 128
buf = np.zeros(slots * 16 * 8, dtype=np.uint64)
assert Lib.sv_debug_bandtime(buf.ctypes.data, slots) == 0
for rep in range(3):
    g = np.random.default_rng(rep)
    r = rng_from_numpy(g)
    st = _native.stats_array(sweeps)
    ctx.band_counts()
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, sweeps, ctypes.byref(r), st, 2), 'run')
    bc = ctx.band_counts()
    buf[:] = 0
    assert Lib.sv_debug_bandtime(buf.ctypes.data, slots) == 0  # (clears nothing: read the last launch's records)
    t = buf.reshape(slots, 16, 8).astype(np.int64)
    busy = t[:, :, 0] > 0
    K = int(busy.any(axis=0).sum())
    t0 = t[:, :, 0][busy].min()
    print(f'[L={L} rep {rep}] band launches {bc}, sweeps per launch {K}, slots with records {int(busy[:, 0].sum())}')
    prev_bar = None
    for j in range(K):
        m = busy[:, j]
        e, b, l0, l1, x, bar = [(t[m, j, i] - t0) * 0.01 for i in range(6)]
        bar_all = (t[t[:, j, 5] > 0, j, 5] - t0) * 0.01
        start = e - (prev_bar if prev_bar is not None else e.min())
        span = bar_all.max() - (prev_bar if prev_bar is not None else e.min())
        print(f'  sweep {j}: WGs {int(m.sum())}  start {np.median(start):5.2f}  bases {np.median(b - e):5.2f}  rows '
              f'{np.median(l0 - b):5.2f}  loop {np.median(l1 - l0):5.2f} (max {np.max(l1 - l0):5.2f})  epi '
              f'{np.median(x - l1):5.2f}  barrier {np.median(bar - x):5.2f}  span {span:6.2f} us')
        prev_bar = bar_all.max()
ctx.check(Lib.sv_villain_destroy(h), 'destroy')
