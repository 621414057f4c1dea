"""A batch of independent Villain NeighborhoodUpdate chains on one GPU (BASELINE config 5).

Replica r is exactly the chain the reference's NeighborhoodUpdate (generator/villain/neighborhood.py:
59-137) produces with `G.rng = rngs[r]`; all replicas advance together, one kernel launch per sweep
(sv_replicas_* in include/supervillain_amd.h).  With inline=True the sweep kernel also measures, for
every replica and sweep, the observables the reference measures inline (observable/observable.py:
50-54): ActionDensity (action.py:25-31), InternalEnergyDensity (energy.py:25-30), WindingSquared
(winding.py:30-37) and TorusWrapping (wrapping.py:17-25).
"""
import ctypes

import numpy as np

from supervillain_amd import _native
from supervillain_amd._abi import SvStats, rngs_from_numpy, rngs_to_numpy

# Default bound on one worm's moves: a worm that never closes (a far-from-equilibrium start can make one) would
# otherwise keep its GPU lane -- and the launch -- running indefinitely.  10^8 moves is ~100x a critical
# L=4096 worm; exceeding it raises (pass max_moves=0 for no bound).
WORM_MAX_MOVES = 100_000_000

# numpy image of sv_stats (include/supervillain_amd.h)
STATS_DTYPE = np.dtype([('accepted', '<i8'), ('proposed', '<i8'), ('acceptance_sum', '<f8'), ('rejections', '<i8')])
assert STATS_DTYPE.itemsize == __import__('ctypes').sizeof(SvStats)


class VillainReplicas:

    def __init__(self, R, N, kappa=0.5, W=1, interval_phi=np.pi, interval_n=1, *, device=None):
        self.R, self.N = int(R), int(N)
        self.kappa, self.W, self.interval_phi, self.interval_n = float(kappa), int(W), float(interval_phi), int(interval_n)
        self.ctx = _native.context(_native.default_device() if device is None else device)
        h = ctypes.c_void_p()
        self.ctx.check(_native.lib().sv_replicas_create(self.ctx.handle, self.R, self.N, ctypes.byref(h)),
                       'sv_replicas_create')
        self.handle = h

    def close(self, _in_del=False):
        if getattr(self, 'handle', None) is not None and _native._LIB is not None:
            h, self.handle = self.handle, None
            _native.destroy(_native._LIB.sv_replicas_destroy, h, 'sv_replicas_destroy', self.ctx, _in_del)

    def __del__(self):
        self.close(_in_del=True)

    def cold(self):
        self.ctx.check(_native.lib().sv_replicas_upload(self.handle, None, None), 'sv_replicas_upload')

    def upload(self, phi, n):
        phi = np.ascontiguousarray(phi, dtype=np.float64).reshape(self.R, self.N, self.N)
        n = np.ascontiguousarray(n, dtype=np.int64).reshape(self.R, 2, self.N, self.N)
        self.ctx.check(_native.lib().sv_replicas_upload(self.handle, _native.ptr(phi), _native.ptr(n)),
                       'sv_replicas_upload')

    def download(self):
        phi = np.empty((self.R, self.N, self.N))
        n = np.empty((self.R, 2, self.N, self.N), dtype=np.int64)
        self.ctx.check(_native.lib().sv_replicas_download(self.handle, _native.ptr(phi), _native.ptr(n)),
                       'sv_replicas_download')
        return phi, n

    def worm(self, rngs, worms=1, max_moves=WORM_MAX_MOVES):
        """`worms` ClassicWorm steps of every replica (supervillain/generator/villain/worm.py:85-183), one GPU
        lane per replica; rngs: R NumPy Generators, advanced in place.  Returns (Vortex_Vortex of each
        replica's last worm (R, N, N) int64, Worm_Length (R, worms) int64)."""
        if len(rngs) != self.R:
            raise ValueError(f'need {self.R} generators')
        r, addrs = rngs_from_numpy(rngs)
        hist = np.zeros((self.R, self.N, self.N), dtype=np.int64)
        lengths = np.zeros((self.R, max(worms, 1)), dtype=np.int64)
        W = 1 if self.W == 1 else 0
        self.ctx.check(_native.lib().sv_replicas_worm_run(self.handle, self.kappa, W, int(worms), int(max_moves), r,
                                                          _native.ptr(hist), _native.ptr(lengths)),
                       'sv_replicas_worm_run')
        rngs_to_numpy(r, rngs, addrs)
        return hist, lengths[:, :worms]

    def run(self, sweeps, rngs, inline=False):
        """`sweeps` sweeps of every replica; rngs: R NumPy Generators, advanced in place.

        Returns (stats, observables): stats has (R, sweeps) arrays 'accepted', 'acceptance' (the
        reference's per-sweep increment of G.acceptance) and 'rejections'; observables is None or a
        dict of (R, sweeps) arrays (TorusWrapping: (R, sweeps, 2))."""
        if len(rngs) != self.R:
            raise ValueError(f'need {self.R} generators')
        r, addrs = rngs_from_numpy(rngs)
        K = max(sweeps, 1)
        st = np.empty((self.R, K), dtype=STATS_DTYPE)  # sv_stats[R][sweeps] (every entry written by the call)
        # the measured arrays are filled by the library's copy-out of each batch, which overlaps the next batch's
        # sweeps (and takes the arrays' first-touch page faults there), instead of NumPy after the call
        acc = np.empty((self.R, K))
        if inline:
            act, energy, w2 = np.empty((self.R, K)), np.empty((self.R, K)), np.empty((self.R, K))
            tw = np.empty((self.R, K, 2), dtype=np.int64)
        else:
            act = energy = w2 = np.empty((self.R, 0))
            tw = np.empty((self.R, 0, 2), dtype=np.int64)
        if inline:
            rc = _native.lib().sv_replicas_run_measured(self.handle, self.kappa, self.W, self.interval_phi,
                                                        self.interval_n, int(sweeps), r, _native.ptr(st),
                                                        _native.ptr(acc), _native.ptr(act), _native.ptr(energy),
                                                        _native.ptr(w2), _native.ptr(tw))
            self.ctx.check(rc, 'sv_replicas_run_measured')
        else:
            self.ctx.check(_native.lib().sv_replicas_run(self.handle, self.kappa, self.W, self.interval_phi,
                                                         self.interval_n, int(sweeps), r, _native.ptr(st), None),
                           'sv_replicas_run')
        rngs_to_numpy(r, rngs, addrs)
        st = st[:, :sweeps]
        if not inline:
            acc = st['acceptance_sum'] / (self.N * self.N)
        stats = {'accepted': st['accepted'], 'acceptance': acc[:, :sweeps], 'rejections': st['rejections']}
        if not inline:
            return stats, None
        return stats, {'ActionDensity': act[:, :sweeps], 'InternalEnergyDensity': energy[:, :sweeps],
                       'WindingSquared': w2[:, :sweeps], 'TorusWrapping': tw[:, :sweeps]}


def worldline_worms(m, v, kappa, W, rngs, worms=1, max_moves=WORM_MAX_MOVES, device=None):
    """`worms` Worldline ClassicWorm steps (supervillain/generator/worldline/worm.py:137-193) of R independent
    chains, one GPU lane each: m (R, 2, N, N) int64 is updated in place, v (R, N, N) int64 (float64 at
    W = infinity) is read.  Returns (Spin_Spin of each chain's last worm (R, N, N), Worm_Length (R, worms))."""
    R, _, N, _ = m.shape
    if m.dtype != np.int64 or not m.flags.c_contiguous:
        raise ValueError('m must be a C-contiguous int64 (R, 2, N, N) array')
    v_float = not (W < float('inf'))
    v = np.ascontiguousarray(v, dtype=np.float64 if v_float else np.int64).reshape(R, N, N)
    if len(rngs) != R:
        raise ValueError(f'need {R} generators')
    W_eff = 2 * np.pi if v_float else float(W)
    ctx = _native.context(_native.default_device() if device is None else device)
    r, addrs = rngs_from_numpy(rngs)
    hist = np.zeros((R, N, N), dtype=np.int64)
    lengths = np.zeros((R, max(worms, 1)), dtype=np.int64)
    ctx.check(_native.lib().sv_worldline_worm_batch(ctx.handle, R, N, float(kappa), W_eff, _native.ptr(m), _native.ptr(v),
                                                    int(v_float), int(worms), int(max_moves), r, _native.ptr(hist),
                                                    _native.ptr(lengths)), 'sv_worldline_worm_batch')
    rngs_to_numpy(r, rngs, addrs)
    return hist, lengths[:, :worms]
