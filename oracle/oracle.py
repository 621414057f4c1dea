"""ctypes front-end to oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see sv_oracle.c's header for the file:line map).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (supervillain_amd) never does.
"""
import ctypes
import os

import numpy as np

from supervillain_amd._abi import SvRng, SvStats, rng_from_numpy, rng_to_numpy

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, 'liboracle.so')
        if not os.path.exists(path):
            raise RuntimeError(f'{path} is missing: run `make -C oracle` (or __graft_entry__.build())')
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        i32, i64, f64, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
        L.sv_o_raw.argtypes = [P(SvRng), i64, vp]
        L.sv_o_uniform.argtypes = [P(SvRng), f64, f64, i64, vp]
        L.sv_o_integers.argtypes = [P(SvRng), ctypes.c_uint32, i64, vp]
        L.sv_o_colors.argtypes = [i32, vp]
        L.sv_o_villain_neighborhood.argtypes = [i32, f64, i64, f64, i64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_villain_neighborhood_rect.argtypes = [i32, i32, f64, i64, f64, i64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_villain_action.argtypes = [i32, f64, vp, vp]
        L.sv_o_villain_action.restype = f64
        L.sv_o_worldline_coexact.argtypes = [i32, f64, f64, i64, vp, vp, i32, i32, P(SvRng), vp]
        L.sv_o_worldline_plaquette_seq.argtypes = [i32, f64, f64, vp, vp, i32, vp, P(SvRng), vp]
        L.sv_o_worldline_plaquette_cb.argtypes = [i32, f64, f64, vp, vp, i32, i32, P(SvRng), vp]
        L.sv_o_villain_site.argtypes = [i32, f64, f64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_villain_link.argtypes = [i32, f64, i64, i64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_villain_exact.argtypes = [i32, f64, i64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_villain_cohomology.argtypes = [i32, f64, i64, vp, vp, i32, P(SvRng), vp]
        L.sv_o_worldline_vortex.argtypes = [i32, f64, f64, i64, vp, vp, i32, i32, P(SvRng), vp]
        L.sv_o_worldline_wrapping.argtypes = [i32, f64, f64, i64, vp, vp, i32, i32, P(SvRng), vp]
        L.sv_o_villain_neighborhood_mt.argtypes = [i32, f64, i64, f64, i64, vp, vp, i32, P(SvRng), vp, i32]
        L.sv_o_villain_worm.argtypes = [i32, f64, i64, vp, vp, i32, P(SvRng), vp, vp]
        L.sv_o_worldline_worm.argtypes = [i32, f64, f64, vp, vp, i32, i32, P(SvRng), vp, vp]
        u32, u64 = ctypes.c_uint32, ctypes.c_uint64
        L.sv_o_philox4x32_10.argtypes = [vp, vp, vp]
        L.sv_o_villain_neighborhood_philox.argtypes = [i32, f64, i64, f64, i64, vp, vp, i32, u64, u64, u32, vp]
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _stats_array(k):
    return (SvStats * max(k, 1))()


def raw(gen, count):
    r = rng_from_numpy(gen)
    out = np.empty(count, dtype=np.uint64)
    lib().sv_o_raw(ctypes.byref(r), count, _ptr(out))
    rng_to_numpy(r, gen)
    return out


def uniform(gen, low, high, count):
    r = rng_from_numpy(gen)
    out = np.empty(count, dtype=np.float64)
    lib().sv_o_uniform(ctypes.byref(r), low, high, count, _ptr(out))
    rng_to_numpy(r, gen)
    return out


def integers(gen, k, count):
    r = rng_from_numpy(gen)
    out = np.empty(count, dtype=np.int64)
    lib().sv_o_integers(ctypes.byref(r), k, count, _ptr(out))
    rng_to_numpy(r, gen)
    return out


def colors(N):
    out = np.empty(N * N, dtype=np.int32)
    ncol = lib().sv_o_colors(N, _ptr(out))
    return ncol, out.reshape(N, N)


def villain_neighborhood(N, kappa, W, phi, n, sweeps, gen, interval_phi=np.pi, interval_n=1):
    """Run `sweeps` NeighborhoodUpdate sweeps in place on (phi (N,N) f64, n (2,N,N) i64)."""
    assert phi.dtype == np.float64 and n.dtype == np.int64
    assert phi.flags.c_contiguous and n.flags.c_contiguous
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    rc = lib().sv_o_villain_neighborhood(N, kappa, int(W), interval_phi, int(interval_n), _ptr(phi), _ptr(n),
                                         sweeps, ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def philox4x32_10(ctr, key):
    """Philox4x32-10 of a 4-word counter under a 2-word key (the optional fast mode's generator)."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.empty(4, dtype=np.uint32)
    lib().sv_o_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def villain_neighborhood_philox(N, kappa, W, phi, n, sweeps, key, counter, interval_phi=np.pi, interval_n=1,
                                thr_override=0):
    """NeighborhoodUpdate sweeps with the counter-based Philox draws (sv_oracle.c's header of that section)."""
    assert phi.dtype == np.float64 and n.dtype == np.int64
    assert phi.flags.c_contiguous and n.flags.c_contiguous
    st = _stats_array(sweeps)
    rc = lib().sv_o_villain_neighborhood_philox(N, kappa, int(W), interval_phi, int(interval_n), _ptr(phi), _ptr(n),
                                                sweeps, key, counter, thr_override, st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    return [st[i] for i in range(sweeps)]


def villain_neighborhood_rect(Nt, Nx, kappa, W, phi, n, sweeps, gen, interval_phi=np.pi, interval_n=1):
    """The same chain on an even Nt x Nx torus (phi (Nt,Nx), n (2,Nt,Nx)); Nt == Nx is the reference's."""
    assert phi.dtype == np.float64 and n.dtype == np.int64
    assert phi.flags.c_contiguous and n.flags.c_contiguous and phi.shape == (Nt, Nx) and n.shape == (2, Nt, Nx)
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    rc = lib().sv_o_villain_neighborhood_rect(Nt, Nx, kappa, int(W), interval_phi, int(interval_n), _ptr(phi), _ptr(n),
                                              sweeps, ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def villain_action(N, kappa, phi, n):
    return lib().sv_o_villain_action(N, kappa, _ptr(phi), _ptr(n))


def worldline_coexact(N, kappa, W_eff, m, v, sweeps, gen, interval_t=1):
    assert m.dtype == np.int64 and m.flags.c_contiguous and v.flags.c_contiguous
    v_is_float = int(v.dtype == np.float64)
    assert v_is_float or v.dtype == np.int64
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    rc = lib().sv_o_worldline_coexact(N, kappa, float(W_eff), int(interval_t), _ptr(m), _ptr(v), v_is_float,
                                      sweeps, ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def worldline_plaquette_seq(N, kappa, W_eff, m, v, order, gen):
    v_is_float = int(v.dtype == np.float64)
    order = np.ascontiguousarray(order, dtype=np.int64)
    r = rng_from_numpy(gen)
    st = _stats_array(1)
    rc = lib().sv_o_worldline_plaquette_seq(N, kappa, float(W_eff), _ptr(m), _ptr(v), v_is_float, _ptr(order),
                                            ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return st[0]


def worldline_plaquette_cb(N, kappa, W_eff, m, v, sweeps, gen):
    v_is_float = int(v.dtype == np.float64)
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    rc = lib().sv_o_worldline_plaquette_cb(N, kappa, float(W_eff), _ptr(m), _ptr(v), v_is_float, sweeps,
                                           ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def villain_generator(kind, N, kappa, W, phi, n, sweeps, gen, interval=None):
    """Run `sweeps` steps of a SURVEY.md 8(f) Villain generator ('SiteUpdate', 'LinkUpdate',
    'ExactUpdate', 'CohomologyUpdate') in place on (phi (N,N) f64, n (2,N,N) i64)."""
    assert phi.dtype == np.float64 and n.dtype == np.int64 and phi.flags.c_contiguous and n.flags.c_contiguous
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    L = lib()
    if kind == 'SiteUpdate':
        rc = L.sv_o_villain_site(N, kappa, np.pi if interval is None else float(interval), _ptr(phi), _ptr(n), sweeps,
                                 ctypes.byref(r), st)
    elif kind == 'LinkUpdate':
        rc = L.sv_o_villain_link(N, kappa, int(W), 1 if interval is None else int(interval), _ptr(phi), _ptr(n), sweeps,
                                 ctypes.byref(r), st)
    elif kind == 'ExactUpdate':
        rc = L.sv_o_villain_exact(N, kappa, 1 if interval is None else int(interval), _ptr(phi), _ptr(n), sweeps,
                                  ctypes.byref(r), st)
    elif kind == 'CohomologyUpdate':
        rc = L.sv_o_villain_cohomology(N, kappa, 1 if interval is None else int(interval), _ptr(phi), _ptr(n), sweeps,
                                       ctypes.byref(r), st)
    else:
        raise ValueError(kind)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def worldline_generator(kind, N, kappa, W_eff, m, v, sweeps, gen, interval=None):
    """Run `sweeps` steps of a SURVEY.md 8(f) Worldline generator ('VortexUpdate' changes v, 'WrappingUpdate'
    changes m) in place on (m (2,N,N) i64, v (N,N) i64, or f64 at W = infinity)."""
    assert m.dtype == np.int64 and m.flags.c_contiguous and v.flags.c_contiguous
    v_is_float = int(v.dtype == np.float64)
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    iv = 1 if interval is None else int(interval)
    fn = {'VortexUpdate': lib().sv_o_worldline_vortex, 'WrappingUpdate': lib().sv_o_worldline_wrapping}[kind]
    rc = fn(N, kappa, float(W_eff), iv, _ptr(m), _ptr(v), v_is_float, sweeps, ctypes.byref(r), st)
    if rc != 0:
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]


def villain_worm(N, kappa, W, phi, n, worms, gen):
    """`worms` Villain ClassicWorm steps in place on n (2,N,N) i64 given phi (N,N) f64.
    Returns (Vortex_Vortex of the last worm (N,N) i64, Worm_Length per worm (worms,) i64)."""
    assert n.dtype == np.int64 and n.flags.c_contiguous
    phi = np.ascontiguousarray(phi, dtype=np.float64)
    r = rng_from_numpy(gen)
    hist = np.zeros((N, N), dtype=np.int64)
    lengths = np.zeros(max(worms, 1), dtype=np.int64)
    W = 0 if W == float('inf') else int(W)  # only W == 1 changes the algorithm
    if lib().sv_o_villain_worm(N, kappa, W, _ptr(phi), _ptr(n), worms, ctypes.byref(r), _ptr(hist), _ptr(lengths)):
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return hist, lengths[:worms]


def worldline_worm(N, kappa, W_eff, m, v, worms, gen):
    """`worms` Worldline ClassicWorm steps in place on m (2,N,N) i64 given v (N,N) (i64, or f64 at W = inf).
    Returns (Spin_Spin of the last worm (N,N) i64, Worm_Length per worm (worms,) i64)."""
    assert m.dtype == np.int64 and m.flags.c_contiguous and v.flags.c_contiguous
    r = rng_from_numpy(gen)
    hist = np.zeros((N, N), dtype=np.int64)
    lengths = np.zeros(max(worms, 1), dtype=np.int64)
    if lib().sv_o_worldline_worm(N, kappa, float(W_eff), _ptr(m), _ptr(v), int(v.dtype == np.float64), worms,
                                 ctypes.byref(r), _ptr(hist), _ptr(lengths)):
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return hist, lengths[:worms]


def villain_neighborhood_mt(N, kappa, W, phi, n, sweeps, gen, threads, interval_phi=np.pi, interval_n=1):
    """villain_neighborhood with the draws and the per-site work split over `threads` OpenMP threads (bench.py's
    multi-core CPU baseline); the same chain as the sequential restatement."""
    assert phi.dtype == np.float64 and n.dtype == np.int64 and phi.flags.c_contiguous and n.flags.c_contiguous
    r = rng_from_numpy(gen)
    st = _stats_array(sweeps)
    if lib().sv_o_villain_neighborhood_mt(N, kappa, W, interval_phi, interval_n, _ptr(phi), _ptr(n), sweeps,
                                          ctypes.byref(r), st, int(threads)):
        raise ValueError('oracle rejected the arguments')
    rng_to_numpy(r, gen)
    return [st[i] for i in range(sweeps)]
