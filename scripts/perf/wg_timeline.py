"""Per-workgroup timeline of villain_sweep_hot (variant built with -DSV_WGTIME=1: entry / loop start / loop end / exit
timestamps from s_memrealtime, 100 MHz, and the hardware ids).  Usage:
  SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so python scripts/perf/wg_timeline.py [single|tile] ...
  (worldline: a variant built with -DSV_WFTIME=1, python scripts/perf/wg_timeline.py worldline [L])"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402
from supervillain_amd.domain import VillainDomain  # noqa: E402

Lib = _native.lib()
if hasattr(Lib, 'sv_debug_wgtime'):  # (variants built with -DSV_WGTIME=1; SV_WFTIME=1 builds have sv_debug_wftime)
    Lib.sv_debug_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int32]


def read(nwg):
    buf = np.zeros(nwg * 6, dtype=np.uint64)
    assert Lib.sv_debug_wgtime(buf.ctypes.data, nwg) == 0
    return buf.reshape(nwg, 6)


def summarize(tag, t, nsx=None):
    idx = np.nonzero(t[:, 0] > 0)[0]
    t = t[idx]
    t0 = t[:, 0].min()
    e, l0, l1, x = [(t[:, i].astype(np.int64) - int(t0)) * 0.01 for i in range(4)]  # us
    hw = t[:, 4] & 0xFFFFFFFF
    xcc = (t[:, 4] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    ncu = len(np.unique(cuid))
    per_cu = np.bincount(np.unique(cuid, return_inverse=True)[1])
    print(f'[{tag}] {len(t)} WGs on {ncu} CUs (WGs per CU: min {per_cu.min()} max {per_cu.max()} mean {per_cu.mean():.2f}); '
          f'span {x.max():.1f} us; entry skew max {e.max():.1f} us (p50 {np.median(e):.1f}); '
          f'prologue p50 {np.median(l0 - e):.1f} p90 {np.percentile(l0 - e, 90):.1f} us; loop p50 {np.median(l1 - l0):.1f} '
          f'p90 {np.percentile(l1 - l0, 90):.1f} max {(l1 - l0).max():.1f} us; epilogue p50 {np.median(x - l1):.1f} us; '
          f'WG lifetime p50 {np.median(x - e):.1f} max {(x - e).max():.1f} us', flush=True)
    loop = l1 - l0
    life = x - e
    tb = (t[:, 5].astype(np.int64) - int(t0)) * 0.01
    print(f'[{tag}] prologue split p50: entry -> row bases {np.median(tb - e):.2f} us, row bases -> loop '
          f'{np.median(l0 - tb):.2f} us', flush=True)
    print(f'[{tag}] loop p50 by XCD: ' + ' '.join(f'{np.median(loop[xcc == k]):.1f}' for k in range(8)) +
          '; exit max by XCD: ' + ' '.join(f'{x[xcc == k].max():.1f}' for k in range(8)), flush=True)
    inv = np.unique(cuid, return_inverse=True)[1]
    wgs_on_cu = per_cu[inv]
    print(f'[{tag}] by WGs on the CU: ' + '; '.join(
        f'{c}: n={int((wgs_on_cu == c).sum())} loop p50 {np.median(loop[wgs_on_cu == c]):.1f} lifetime p50 '
        f'{np.median(life[wgs_on_cu == c]):.1f} last exit {x[wgs_on_cu == c].max():.1f}'
        for c in np.unique(wgs_on_cu)), flush=True)
    for c in np.unique(wgs_on_cu):
        cus = np.unique(inv[wgs_on_cu == c])
        ranks = np.array([np.sort(life[inv == u]) for u in cus])
        ends = np.array([x[inv == u].max() for u in cus])
        print(f'[{tag}] CUs with {c} WGs: lifetime by rank within the CU ' +
              ' '.join(f'{v:.1f}' for v in ranks.mean(axis=0)) +
              f'; CU finish p10 {np.percentile(ends, 10):.1f} p50 {np.median(ends):.1f} max {ends.max():.1f}', flush=True)
    # occupancy over time: WGs resident (entry..exit) in 2-us bins
    bins = np.arange(0, x.max() + 2, 2.0)
    occ = [int(((e <= b) & (x > b)).sum()) for b in bins]
    print(f'[{tag}] resident WGs every 2 us: {occ}', flush=True)
    if nsx:
        # logical strip index of each launch slot (hot_body's XCD-aware mapping), its column strip
        G = len(idx)
        per, rem = G // 8, G % 8
        xcd_, k_ = idx & 7, idx >> 3
        b = xcd_ * per + np.minimum(xcd_, rem) + k_
        ix = b % nsx
        loop = l1 - l0
        by_ix = [float(np.mean(loop[ix == i])) for i in range(nsx)]
        print(f'[{tag}] loop us by column strip: ' + ' '.join(f'{v:.0f}' for v in by_ix), flush=True)
        order = np.argsort(e)
        thirds = np.array_split(order, 4)
        print(f'[{tag}] loop us by dispatch quarter: ' + ' '.join(f'{np.mean(loop[q]):.1f}' for q in thirds) +
              f'; lifetime by quarter: ' + ' '.join(f'{np.mean((x - e)[q]):.1f}' for q in thirds), flush=True)


mode = sys.argv[1] if len(sys.argv) > 1 else 'single'
ctx = _native.context(0)
if mode == 'worldline':
    # config 3's worldline_step_fused (variant built with -DSV_WFTIME=1): the last launch of each call of 50 steps
    Lib.sv_debug_wftime.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, L, 0, ctypes.byref(h)), 'create')
    m, v = np.zeros((2, L, L), dtype=np.int64), np.zeros((L, L), dtype=np.int64)
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'upload')
    r = rng_from_numpy(np.random.default_rng(0))
    st = _native.stats_array(2 * 50)
    for k in range(4):
        ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, 0.5, 1.0, 1, 50, ctypes.byref(r), st), 'run')
        buf = np.zeros(65536 * 6, dtype=np.uint64)
        assert Lib.sv_debug_wftime(buf.ctypes.data, 65536) == 0
        t = buf.reshape(65536, 6)
        summarize(f'worldline L={L} call {k}', t)
        # per strip: worldline_step_fused's XCD-aware slot -> strip mapping, nsx = ceil(L / 119) column strips
        nsx = (L + 118) // 119
        idx = np.nonzero(t[:, 0] > 0)[0]
        G = len(idx)
        per, rem = G // 8, G % 8
        b = (idx & 7) * per + np.minimum(idx & 7, rem) + (idx >> 3)
        nsy = (L + 40) // 41
        ni = nsx - 1
        tail = G == ni * (nsy + 1) + (L + 24) // 25  # the turned layout with the last row strip cut in two
        turned = tail or G == ni * nsy + (L + 24) // 25
        t0 = np.zeros(G, dtype=np.int64)
        th = np.full(G, 41)
        if turned:
            ny = nsy - 1 if tail else nsy
            ix = np.where(b < ni * ny, 1 + b % ni, 0)
            t0 = np.where(b < ni * ny, (b // ni) * 41, 0)
            if tail:
                kk = b - ni * ny
                inr = (b >= ni * ny) & (b < ni * (ny + 2))
                half = (L - ny * 41 + 1) // 2
                ix = np.where(inr, 1 + kk % ni, ix)
                t0 = np.where(inr, ny * 41 + (kk // ni) * half, t0)
                th = np.where(inr, half, th)
            seam = b >= ni * (ny + 2 if tail else ny)
            t0 = np.where(seam, (b - ni * (ny + 2 if tail else ny)) * 25, t0)
            th = np.where(seam, 25, th)
        else:
            ix, t0 = b % nsx, (b // nsx) * 41
        t1 = np.minimum(t0 + th, L)
        iy = t0  # (printed as the strip's first row)
        tt = t[idx]
        t0_ = int(tt[:, 0].min())
        e, l0, l1, x = [(tt[:, i].astype(np.int64) - t0_) * 0.01 for i in range(4)]
        edge = (ix == 0) | ((ix == nsx - 1) & (not turned))
        redge = (t0 == 0) | (t1 == L)
        for nm, sel in (('interior', ~edge & ~redge), ('seam columns', edge & ~redge), ('seam rows', ~edge & redge),
                        ('corners', edge & redge)):
            if sel.any():
                print(f'[worldline L={L} call {k}] {nm}: n={int(sel.sum())} loop p50 {np.median((l1 - l0)[sel]):.1f} '
                      f'max {(l1 - l0)[sel].max():.1f}; prologue p50 {np.median((l0 - e)[sel]):.2f} (to bases '
                      f'{np.median(((tt[:, 5].astype(np.int64) - t0_) * 0.01 - e)[sel]):.2f}); epilogue p50 '
                      f'{np.median((x - l1)[sel]):.2f}; exit p50 {np.median(x[sel]):.1f} max {x[sel].max():.1f}', flush=True)
        last = np.argsort(x)[-8:]
        print(f'[worldline L={L} call {k}] last exits (ix, first row, xcd, entry, loop, exit): ' + ' '.join(
            f'({ix[j]},{iy[j]},{int((tt[j, 4] >> 32) & 0xF)},{e[j]:.1f},{(l1 - l0)[j]:.1f},{x[j]:.1f})' for j in last),
            flush=True)
    sys.exit(0)
if mode == 'single':
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
    r = rng_from_numpy(np.random.default_rng(0))
    st = _native.stats_array(64)
    for k in range(4):
        ctx.check(Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, 1, ctypes.byref(r), st, 2), 'run')
        summarize(f'L={L} sweep {k}', read(65536), nsx=(L + 122) // 123)
else:
    Nt, Nx = int(sys.argv[2]), int(sys.argv[3])
    dom = VillainDomain(Nt, Nx, (1, 1), 0.5, 1)
    dom.cold()
    g = np.random.default_rng(0)
    for k in range(3):
        dom.run(4, g)  # the last launch of a 4-sweep group decides exactly the tile
        summarize(f'tile {Nt}x{Nx} group {k}', read(65536), nsx=(Nx + 122) // 123)
    dom.close()
