"""Per-workgroup timeline of the split replay (villain_sweep_hot_split) against a plain hot sweep, L=4096, from a variant
built with -DSV_WGTIME=1:
  bash scripts/build_variant.sh wgtime -DSV_WGTIME=1
  SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so python scripts/perf/split_timeline.py [rank_frac]
A crafted PCG64 state forces a NumPy Lemire rejection in colour 0's second choice block at rank rank_frac * V/2, in
the call's only sweep: the hot sweep aborts, and the call's last launch is the split replay, whose g_wgtime entries are
read back (then one clean sweep for comparison)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402
from tests.golden import crafted_generator  # noqa: E402

Lib = _native.lib()
Lib.sv_debug_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int32]
N = 4096
V = N * N
frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.37
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, N, ctypes.byref(h)), 'create')
phi = np.zeros((N, N))
n = np.zeros((2, N, N), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
st = _native.stats_array(64)
NWG = 4096


def run(gen, k):
    r = rng_from_numpy(gen)
    ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(r), st, 2), 'run')


def timeline(tag):
    buf = np.zeros(NWG * 6, dtype=np.uint64)
    assert Lib.sv_debug_wgtime(buf.ctypes.data, NWG) == 0
    t = buf.reshape(NWG, 6)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    e, l0, l1, x = [(t[:, i].astype(np.int64) - int(t0)) * 0.01 for i in range(4)]
    d = x - e
    o = np.argsort(-x)[:8]
    print(f'[{tag}] {len(t)} WGs, span {x.max():.1f} us, lifetime p50 {np.median(d):.1f} us max {d.max():.1f}; '
          f'last exits: ' + ', '.join(f'{x[i]:.1f} (entry {e[i]:.1f}, life {d[i]:.1f})' for i in o), flush=True)
    q = np.percentile(d, [10, 25, 50, 75, 90, 99])
    ds = np.sort(d)[::-1]
    print(f'    lifetime sum {d.sum() / 1e3:.2f} ms; p10..p99 ' + ' '.join(f'{v:.1f}' for v in q) +
          '; top 40 ' + ' '.join(f'{v:.0f}' for v in ds[:40]), flush=True)


for rep in range(3):
    rank = int(frac * V / 2) + 1000 * rep
    w = V + V // 2 + V // 4 + rank // 2  # colour 0, block 1 (bwd, mu = 0), has = 0
    run(np.random.default_rng(5), 3)  # warm
    g = crafted_generator(17 + rep, w, rank % 2)
    ctx.sweep_counts()
    ctx.split_counts()
    run(g, 1)
    print('split sweeps', ctx.split_counts(), ctx.sweep_counts())
    timeline(f'split rank {rank}')
    run(np.random.default_rng(rep), 1)
    timeline('hot')
Lib.sv_villain_destroy(h)
