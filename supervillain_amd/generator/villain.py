"""NeighborhoodUpdate on the MI355X: supervillain/generator/villain/neighborhood.py:12-149.

Same constructor, attributes (`rng`, `accepted`, `proposed`, `acceptance`, `sweeps`), `step` contract
and `report()` text as the reference.  The sweep itself runs in libsvhip.so
(`sv_villain_run`, include/supervillain_amd.h); `self.rng` is a NumPy Generator(PCG64) whose stream
the device replays, so `G.rng = np.random.default_rng(seed)` gives the reference's chain.
"""
import ctypes

import numpy as np

from supervillain_amd import _native
from supervillain_amd.batch import Batch
from supervillain_amd.generator._common import DeviceState, rng_from_numpy, rng_to_numpy, wrap_like
from supervillain_amd.generator.generator import Generator


def _is_villain(action):
    return type(action).__name__ == 'Villain' and hasattr(action, 'kappa') and hasattr(action, 'Lattice')


class NeighborhoodUpdate(DeviceState, Generator):
    r'''Checkerboard Metropolis sweep of phi and the 2D links around each site (neighborhood.py:12-36).

    Extra keyword-only arguments (not in the reference):
      device: HIP device ordinal (default: $SV_DEVICE, $LOCAL_RANK, else 0).
      inline: also return ActionDensity, InternalEnergyDensity, WindingSquared and TorusWrapping of
              each new configuration, reduced on the device (measured inline, observable.py:50-54).
      path:   0 auto (fused sweep kernel for even N), 1 per-colour kernels, 2 fused only.
    '''

    INLINE = ('ActionDensity', 'InternalEnergyDensity', 'WindingSquared', 'TorusWrapping')

    def __init__(self, action, interval_phi=np.pi, interval_n=1, *, device=None, inline=False, path=0):
        if not _is_villain(action):
            raise ValueError('The Neighborhood Metropolis update requires the Villain action.')
        self.Action = action
        self.Lattice = action.Lattice
        self.kappa = action.kappa
        self.interval_phi = interval_phi
        self.interval_n = interval_n
        self.rng = np.random.default_rng()
        self.n_changes = np.arange(-interval_n, 1 + interval_n)
        self.accepted = 0
        self.proposed = 0
        self.acceptance = 0.
        self.sweeps = 0
        self.device = device
        self.inline = inline
        self.path = path

    def __str__(self):
        return 'NeighborhoodUpdate'

    # -------------------------------------------------------------------------------- device
    def _state(self):
        L = self.Lattice
        if L.D != 2:
            raise NotImplementedError('the MI355X NeighborhoodUpdate is implemented for D=2 lattices')
        W = self.Action.W
        if not (np.isfinite(W) and float(W) == int(W)):
            raise NotImplementedError('NeighborhoodUpdate needs a finite integer W (W * choice(...) must be an int)')
        dev = self.__dict__.get('_dev')
        if dev is None or dev[1] != L.N:
            ctx = self._device_context()
            h = ctypes.c_void_p()
            ctx.check(_native.lib().sv_villain_create(ctx.handle, L.N, ctypes.byref(h)), 'sv_villain_create')
            dev = (ctx, L.N, h)
            self._dev = dev
        return dev

    def __del__(self):
        dev = self.__dict__.get('_dev')
        if dev is not None and _native._LIB is not None:
            try:
                _native._LIB.sv_villain_destroy(dev[2])
            except Exception:
                pass

    def _advance(self, phi, n, sweeps):
        """Run `sweeps` sweeps on host arrays phi (1,N,N) f64 and n (2,N,N) i64, in place."""
        ctx, N, h = self._state()
        L = _native.lib()
        st = _native.stats_array(sweeps)
        r = rng_from_numpy(self.rng)
        ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_upload')
        ctx.check(L.sv_villain_run(h, float(self.kappa), int(self.Action.W), float(self.interval_phi),
                                   int(self.interval_n), sweeps, ctypes.byref(r), st, int(self.path)),
                  'sv_villain_run')
        inline = None
        if self.inline:
            out = np.zeros(4)
            ctx.check(L.sv_villain_observables(h, float(self.kappa), _native.ptr(out)), 'sv_villain_observables')
            inline = out
        ctx.check(L.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_download')
        rng_to_numpy(r, self.rng)
        V = self.Lattice.sites
        for k in range(sweeps):  # fold exactly like neighborhood.py:131-135
            self.sweeps += 1
            self.proposed += V
            self.acceptance += st[k].acceptance_sum / V
            self.accepted += int(st[k].accepted)
        return inline

    def _result(self, cfg, phi, n, inline):
        L = self.Lattice
        out = cfg | {'phi': wrap_like(cfg['phi'], phi, 0, L), 'n': wrap_like(cfg['n'], n, 1, L)}
        if inline is not None:
            V, kappa = L.sites, self.kappa
            S = inline[0]
            out |= {
                'ActionDensity': S / V,                                   # observable/action.py:25-31
                'InternalEnergyDensity': S / (V * kappa),                 # observable/energy.py:25-30
                'WindingSquared': inline[1] / L.cells_of_degree[2],       # observable/winding.py:30-37
                'TorusWrapping': np.array([int(round(inline[2])), int(round(inline[3]))], dtype=np.int64),
            }
        return out

    def _fields(self, cfg):
        N = self.Lattice.N
        phi = np.array(cfg['phi'], dtype=np.float64, order='C', copy=True).reshape(1, N, N)
        n = np.array(cfg['n'], dtype=np.int64, order='C', copy=True).reshape(2, N, N)
        return phi, n

    # -------------------------------------------------------------------------------- protocol
    def step(self, cfg):
        r'''One sweep: every site proposes phi += U(-interval_phi, interval_phi) and W*{-n..n} on its 2D
        links, colour by colour (neighborhood.py:59-137).  The input is not mutated.'''
        phi, n = self._fields(cfg)
        inline = self._advance(phi, n, 1)
        return self._result(cfg, phi, n, inline)

    def _steps(self, cfg, count):
        """`count` consecutive steps in one device call (used by KeepEvery)."""
        phi, n = self._fields(cfg)
        inline = self._advance(phi, n, count)
        return self._result(cfg, phi, n, inline)

    def inline_observables(self, steps):
        if not self.inline:
            return dict()
        return {
            'ActionDensity': Batch(steps, shape=(), dtype=float),
            'InternalEnergyDensity': Batch(steps, shape=(), dtype=float),
            'WindingSquared': Batch(steps, shape=(), dtype=float),
            'TorusWrapping': Batch(steps, shape=(self.Lattice.D,), dtype=int),
        }

    def report(self):
        return (
            f'There were {self.accepted} neighborhood proposals accepted of {self.proposed} proposed updates.'
            + '\n' +
            f'    {self.accepted/self.proposed:.6f} acceptance rate'
            + '\n' +
            f'    {self.acceptance / self.sweeps:.6f} average Metropolis acceptance probability.'
        )
