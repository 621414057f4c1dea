"""A batch of independent Villain NeighborhoodUpdate chains on one GPU (BASELINE config 5).

Replica r is exactly the chain the reference's NeighborhoodUpdate (generator/villain/neighborhood.py:
59-137) produces with `G.rng = rngs[r]`; all replicas advance together, one kernel launch per sweep
(sv_replicas_* in include/supervillain_amd.h).  With inline=True the sweep kernel also measures, for
every replica and sweep, the observables the reference measures inline (observable/observable.py:
50-54): ActionDensity (action.py:25-31), InternalEnergyDensity (energy.py:25-30), WindingSquared
(winding.py:30-37) and TorusWrapping (wrapping.py:17-25).
"""
import ctypes
import threading

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
    """R replicas of an N x N Villain lattice in HBM.  streams > 1 (default: 2 from 256 replicas on) keeps them as that
    many part-batches, each on a HIP stream of its own (its own sv_ctx) driven by its own host thread, so that one
    part's launch tails and batch boundaries overlap the other's sweeps (config 5: +11-16% measured).  The
    results are the same bit for bit as one batch's -- the statistics and inline observables are exact sums, whatever
    the replica count of a launch (supervillain_amd/csrc/common.h; tests/test_gpu_observables.py)."""

    def __init__(self, R, N, kappa=0.5, W=1, interval_phi=np.pi, interval_n=1, *, device=None, streams=None):
        self.R, self.N = int(R), int(N)
        self.kappa, self.W, self.interval_phi, self.interval_n = float(kappa), int(W), float(interval_phi), int(interval_n)
        device = _native.default_device() if device is None else device
        streams = (2 if self.R >= 256 else 1) if streams is None else max(1, min(int(streams), self.R))
        self.ctx = _native.context(device)
        self.parts = []  # (first replica, count, context, handle)
        first = 0
        for i in range(streams):
            count = self.R // streams + (1 if i < self.R % streams else 0)
            ctx = self.ctx if i == 0 else _native.Context(device)  # (a stream of its own)
            h = ctypes.c_void_p()
            ctx.check(_native.lib().sv_replicas_create(ctx.handle, count, self.N, ctypes.byref(h)),
                      'sv_replicas_create')
            self.parts.append((first, count, ctx, h))
            first += count
        self.handle = self.parts[0][3] if len(self.parts) == 1 else None  # (the C-ABI handle of a one-part batch)

    @property
    def contexts(self):
        return [p[2] for p in self.parts]

    def close(self, _in_del=False):
        parts, self.parts = getattr(self, 'parts', []), []
        self.handle = None
        err = None
        for _, _, ctx, h in parts:
            if h is not None and _native._LIB is not None:
                try:
                    _native.destroy(_native._LIB.sv_replicas_destroy, h, 'sv_replicas_destroy', ctx, _in_del)
                except _native.NativeError as e:
                    err = err or e
        if err is not None:
            raise err

    def __del__(self):
        self.close(_in_del=True)

    def _each(self, fn):
        """fn(first, count, ctx, handle) for every part: the later parts on their own threads, the first on this one
        (ctypes releases the GIL inside the library); re-raises the first failure after every part has returned."""
        if len(self.parts) == 1:
            return [fn(*self.parts[0])]
        out = [None] * len(self.parts)
        errs = [None] * len(self.parts)

        def work(i):
            try:
                out[i] = fn(*self.parts[i])
            except BaseException as e:  # (joined below)
                errs[i] = e
        threads = [threading.Thread(target=work, args=(i,)) for i in range(1, len(self.parts))]
        for t in threads:
            t.start()
        work(0)
        for t in threads:
            t.join()
        for e in errs:
            if e is not None:
                raise e
        return out

    def cold(self):
        for _, _, ctx, h in self.parts:
            ctx.check(_native.lib().sv_replicas_upload(h, None, None), 'sv_replicas_upload')

    def upload(self, phi, n):
        phi = np.ascontiguousarray(phi, dtype=np.float64).reshape(self.R, self.N, self.N)
        n = np.ascontiguousarray(n, dtype=np.int64).reshape(self.R, 2, self.N, self.N)
        for a, c, ctx, h in self.parts:
            ctx.check(_native.lib().sv_replicas_upload(h, _native.ptr(phi[a:a + c]), _native.ptr(n[a:a + c])),
                      'sv_replicas_upload')

    def download(self):
        phi = np.empty((self.R, self.N, self.N))
        n = np.empty((self.R, 2, self.N, self.N), dtype=np.int64)
        for a, c, ctx, h in self.parts:
            ctx.check(_native.lib().sv_replicas_download(h, _native.ptr(phi[a:a + c]), _native.ptr(n[a:a + c])),
                      'sv_replicas_download')
        return phi, n

    def worm(self, rngs, worms=1, max_moves=WORM_MAX_MOVES):
        """`worms` ClassicWorm steps of every replica (supervillain/generator/villain/worm.py:85-183), one GPU
        lane per replica; rngs: R NumPy Generators, advanced in place.  Returns (Vortex_Vortex of each
        replica's last worm (R, N, N) int64, Worm_Length (R, worms) int64)."""
        if len(rngs) != self.R:
            raise ValueError(f'need {self.R} generators')
        hist = np.zeros((self.R, self.N, self.N), dtype=np.int64)
        lengths = np.zeros((self.R, max(worms, 1)), dtype=np.int64)
        W = 1 if self.W == 1 else 0

        def part(a, c, ctx, h):
            r, addrs = rngs_from_numpy(rngs[a:a + c])
            ctx.check(_native.lib().sv_replicas_worm_run(h, self.kappa, W, int(worms), int(max_moves), r,
                                                         _native.ptr(hist[a:a + c]), _native.ptr(lengths[a:a + c])),
                      'sv_replicas_worm_run')
            rngs_to_numpy(r, rngs[a:a + c], addrs)
        self._each(part)
        return hist, lengths[:, :worms]

    def run(self, sweeps, rngs, inline=False):
        """`sweeps` sweeps of every replica; rngs: R NumPy Generators, advanced in place.

        Returns (stats, observables): stats has (R, sweeps) arrays 'accepted', 'acceptance' (the
        reference's per-sweep increment of G.acceptance) and 'rejections'; observables is None or a
        dict of (R, sweeps) arrays (TorusWrapping: (R, sweeps, 2))."""
        if len(rngs) != self.R:
            raise ValueError(f'need {self.R} generators')
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

        def part(a, c, ctx, h):  # (row blocks of the result arrays: contiguous)
            r, addrs = rngs_from_numpy(rngs[a:a + c])
            b = slice(a, a + c)
            if inline:
                rc = _native.lib().sv_replicas_run_measured(h, self.kappa, self.W, self.interval_phi, self.interval_n,
                                                            int(sweeps), r, _native.ptr(st[b]), _native.ptr(acc[b]),
                                                            _native.ptr(act[b]), _native.ptr(energy[b]),
                                                            _native.ptr(w2[b]), _native.ptr(tw[b]))
                ctx.check(rc, 'sv_replicas_run_measured')
            else:
                ctx.check(_native.lib().sv_replicas_run(h, self.kappa, self.W, self.interval_phi, self.interval_n,
                                                        int(sweeps), r, _native.ptr(st[b]), None), 'sv_replicas_run')
            rngs_to_numpy(r, rngs[a:a + c], addrs)
        self._each(part)
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
