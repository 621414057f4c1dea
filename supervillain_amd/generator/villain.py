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
from supervillain_amd.replicas import WORM_MAX_MOVES


def _is_villain(action):
    return type(action).__name__ == 'Villain' and hasattr(action, 'kappa') and hasattr(action, 'Lattice')


class NeighborhoodUpdate(DeviceState, Generator):
    r'''Checkerboard Metropolis sweep of phi and the 2D links around each site (neighborhood.py:12-36).

    Extra keyword-only arguments (not in the reference):
      device: HIP device ordinal (default: $SV_DEVICE, $LOCAL_RANK, else 0).
      inline: also return ActionDensity, InternalEnergyDensity, WindingSquared and TorusWrapping of
              each new configuration, reduced on the device (measured inline, observable.py:50-54).
      path:   0 auto (fused sweep kernel for even N), 1 per-colour kernels, 2 fused only.
      philox: an integer seed selects the optional counter-based mode (SURVEY.md 8(b) sv_rng mode 1): every draw
              comes from Philox4x32-10 by (site, sweep, slot) under that key instead of from `rng` -- a different,
              statistically equivalent chain with no NumPy-rejection replays (sv_villain_run_philox).  The sweep
              counter is `philox_counter`.
    '''

    INLINE = ('ActionDensity', 'InternalEnergyDensity', 'WindingSquared', 'TorusWrapping')

    def __init__(self, action, interval_phi=np.pi, interval_n=1, *, device=None, inline=False, path=0, philox=None):
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
        self.philox = philox
        self.philox_counter = 0

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
            self._dev = None
            _native.destroy(_native._LIB.sv_villain_destroy, dev[2], 'sv_villain_destroy (' + type(self).__name__ + ')',
                            dev[0], in_del=True)

    DEVICE_KIND = 'villain'

    def _run_on(self, ctx, h, sweeps):
        """`sweeps` sweeps on the device-resident state h (sv_villain); folds the counters like
        neighborhood.py:131-135 and returns the inline observables of the new state (or None)."""
        L = _native.lib()
        st = _native.stats_array(sweeps)
        if self.__dict__.get('philox') is not None:
            from supervillain_amd._abi import SvPhilox
            ph = SvPhilox(int(self.philox) & ((1 << 64) - 1), int(self.philox_counter), 0)
            ctx.check(L.sv_villain_run_philox(h, float(self.kappa), int(self.Action.W), float(self.interval_phi),
                                              int(self.interval_n), sweeps, ctypes.byref(ph), st),
                      'sv_villain_run_philox')
            self.philox_counter = int(ph.counter)
        else:
            r = rng_from_numpy(self.rng)
            ctx.check(L.sv_villain_run(h, float(self.kappa), int(self.Action.W), float(self.interval_phi),
                                       int(self.interval_n), sweeps, ctypes.byref(r), st, int(self.path)),
                      'sv_villain_run')
            rng_to_numpy(r, self.rng)
        V = self.Lattice.sites

        def fold():
            for k in range(sweeps):
                self.sweeps += 1
                self.proposed += V
                self.acceptance += st[k].acceptance_sum / V
                self.accepted += int(st[k].accepted)
        ctx.fold_later(fold)
        if self.inline:
            out = np.zeros(4)
            ctx.check(L.sv_villain_observables(h, float(self.kappa), _native.ptr(out)), 'sv_villain_observables')
            return out
        return None

    def _advance(self, phi, n, sweeps):
        """Run `sweeps` sweeps on host arrays phi (1,N,N) f64 and n (2,N,N) i64, in place."""
        ctx, N, h = self._state()
        L = _native.lib()
        ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_upload')
        inline = self._run_on(ctx, h, sweeps)
        ctx.check(L.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_download')
        return inline

    def _inline_dict(self, inline):
        L = self.Lattice
        V, kappa = L.sites, self.kappa
        S = inline[0]
        return {
            'ActionDensity': S / V,                                   # observable/action.py:25-31
            'InternalEnergyDensity': S / (V * kappa),                 # observable/energy.py:25-30
            'WindingSquared': inline[1] / L.cells_of_degree[2],       # observable/winding.py:30-37
            'TorusWrapping': np.array([int(round(inline[2])), int(round(inline[3]))], dtype=np.int64),
        }

    def _result(self, cfg, phi, n, inline):
        L = self.Lattice
        out = cfg | {'phi': wrap_like(cfg['phi'], phi, 0, L), 'n': wrap_like(cfg['n'], n, 1, L)}
        if inline is not None:
            out |= self._inline_dict(inline)
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


# ------------------------------------------------------------------------------------------------
# The rest of the Villain Hammer's local updates: SiteUpdate, LinkUpdate, ExactUpdate,
# CohomologyUpdate.  Same constructors, attributes, `step` contract and `report()` text as the
# reference; each sweep runs in libsvhip.so on a device-resident (phi, n).

class _VillainLocal(DeviceState, Generator):
    """Shared plumbing: device state, host<->device copies and the reference's counter folding."""

    NAME = None
    NOUN = None                 # report() wording
    RETURNS = ('phi', 'n')      # fields the step changes (the rest of cfg passes through)

    def _init_common(self, action, device):
        if not _is_villain(action):
            raise ValueError('Need a Villain action')
        self.Action = action
        self.Lattice = action.Lattice
        self.kappa = action.kappa
        self.rng = np.random.default_rng()
        self.accepted = 0
        self.proposed = 0
        self.acceptance = 0.
        self.sweeps = 0
        self.device = device

    def __str__(self):
        return self.NAME

    def _state(self):
        L = self.Lattice
        if L.D != 2:
            raise NotImplementedError(f'the MI355X {self.NAME} is implemented for D=2 lattices')
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
            self._dev = None
            _native.destroy(_native._LIB.sv_villain_destroy, dev[2], 'sv_villain_destroy (' + type(self).__name__ + ')',
                            dev[0], in_del=True)

    def _proposals(self):
        return self.Lattice.sites

    DEVICE_KIND = 'villain'

    def _run_on(self, ctx, h, sweeps):
        """`sweeps` steps on the device-resident state h (sv_villain), counters folded like the reference."""
        L = _native.lib()
        st = _native.stats_array(sweeps)
        r = rng_from_numpy(self.rng)
        ctx.check(self._run(L, h, sweeps, r, st), f'{self.NAME} run')
        rng_to_numpy(r, self.rng)
        P = self._proposals()

        def fold():
            for k in range(sweeps):
                self.sweeps += 1
                self.proposed += P
                self.acceptance += st[k].acceptance_sum / P
                self.accepted += int(st[k].accepted)
        ctx.fold_later(fold)
        return None

    def _advance(self, phi, n, sweeps):
        ctx, N, h = self._state()
        L = _native.lib()
        ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_upload')
        self._run_on(ctx, h, sweeps)
        ctx.check(L.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_download')

    def _fields(self, cfg):
        N = self.Lattice.N
        phi = np.array(cfg['phi'], dtype=np.float64, order='C', copy=True).reshape(1, N, N)
        n = np.array(cfg['n'], dtype=np.int64, order='C', copy=True).reshape(2, N, N)
        return phi, n

    def _result(self, cfg, phi, n):
        L = self.Lattice
        new = {'phi': wrap_like(cfg['phi'], phi, 0, L), 'n': wrap_like(cfg['n'], n, 1, L)}
        return cfg | {k: new[k] for k in self.RETURNS}

    def step(self, cfg):
        phi, n = self._fields(cfg)
        self._advance(phi, n, 1)
        return self._result(cfg, phi, n)

    def _steps(self, cfg, count):
        """`count` consecutive steps in one device call (used by KeepEvery)."""
        phi, n = self._fields(cfg)
        self._advance(phi, n, count)
        return self._result(cfg, phi, n)

    def inline_observables(self, steps):
        return {}

    def report(self):
        return (
            f'There were {self.accepted} {self.NOUN} proposals accepted of {self.proposed} proposed updates.'
            + '\n' +
            f'    {self.accepted/self.proposed:.6f} acceptance rate'
            + '\n' +
            f'    {self.acceptance / self.sweeps:.6f} average Metropolis acceptance probability.'
        )


class SiteUpdate(_VillainLocal):
    r'''Checkerboard Metropolis update of phi alone, n untouched (supervillain/generator/villain/site.py:12-135):
    Δφ_x ~ U(-interval_phi, +interval_phi) on one colour at a time.'''

    NAME = 'SiteUpdate'
    NOUN = 'single-phi'
    RETURNS = ('phi',)

    def __init__(self, action, interval_phi=np.pi, *, device=None):
        self._init_common(action, device)
        self.interval_phi = interval_phi

    def _run(self, L, h, sweeps, r, st):
        return L.sv_villain_site_run(h, float(self.kappa), float(self.interval_phi), sweeps, ctypes.byref(r), st)


class LinkUpdate(_VillainLocal):
    r'''Independent Metropolis updates of every link, Δn ~ W × {-interval_n..-1, 1..interval_n}
    (supervillain/generator/villain/link.py:12-109).'''

    NAME = 'LinkUpdate'
    NOUN = 'single-link'
    RETURNS = ('n',)

    def __init__(self, action, interval_n=1, *, device=None):
        self._init_common(action, device)
        W = action.W
        if not (np.isfinite(W) and float(W) == int(W)):
            raise NotImplementedError('LinkUpdate needs a finite integer W (W * choice(...) is an integer change)')
        self.interval_n = interval_n
        self.n_changes = tuple(n for n in range(-interval_n, 0)) + tuple(n for n in range(1, interval_n + 1))

    def _proposals(self):
        return 2 * self.Lattice.sites  # int(np.prod(n.shape)), link.py:95

    def _run(self, L, h, sweeps, r, st):
        return L.sv_villain_link_run(h, float(self.kappa), int(self.Action.W), int(self.interval_n), sweeps,
                                     ctypes.byref(r), st)


class ExactUpdate(_VillainLocal):
    r'''Checkerboard Metropolis update n -> n + dz with an integer zero-form z_x ~ {-interval_z..-1, 1..interval_z},
    which keeps dn unchanged (supervillain/generator/villain/exact.py:12-137).'''

    NAME = 'ExactUpdate'
    NOUN = 'exact'
    RETURNS = ('n',)

    def __init__(self, action, interval_z=1, *, device=None):
        self._init_common(action, device)
        self.interval_z = interval_z
        self.zs = tuple(z for z in range(-interval_z, 0)) + tuple(z for z in range(1, interval_z + 1))

    def _run(self, L, h, sweeps, r, st):
        return L.sv_villain_exact_run(h, float(self.kappa), int(self.interval_z), sweeps, ctypes.byref(r), st)


class CohomologyUpdate(_VillainLocal):
    r'''Winding-sector update: per direction mu, n_mu += h_mu on the slice x_mu = 0, h_mu ~ {-interval_h..-1,
    1..interval_h}, Metropolized as one proposal (supervillain/generator/villain/cohomology.py:12-125).'''

    NAME = 'CohomologyUpdate'
    NOUN = 'cohomology'
    RETURNS = ('n',)

    def __init__(self, action, interval_h=1, *, device=None):
        self._init_common(action, device)
        self.interval_h = interval_h
        self.h = tuple(h for h in range(-interval_h, 0)) + tuple(h for h in range(1, interval_h + 1))

    def _proposals(self):
        return self.Lattice.D

    def _run(self, L, h, sweeps, r, st):
        return L.sv_villain_cohomology_run(h, float(self.kappa), int(self.interval_h), sweeps, ctypes.byref(r), st)


# ------------------------------------------------------------------------------------------------
# the ClassicWorm.

def _worm_report(lengths):
    l = np.array(lengths)
    return f'There were {len(l)} worms.\nWorms lengths:\n    mean {l.mean()}\n    std  {l.std()}\n    max  {max(l)}'


class ClassicWorm(DeviceState, Generator):
    r'''The Prokof'ev-Svistunov worm on the Villain links (supervillain/generator/villain/worm.py:17-131):
    head and tail on plaquettes, the head crosses links changing n by ±1, and the displacement histogram of
    every move is the inline ``Vortex_Vortex`` measurement.  A worm is a sequential walk, so the device runs
    one chain per GPU lane (``sv_villain_worm_run``); batches of chains use
    :meth:`supervillain_amd.replicas.VillainReplicas.worm`.  ``max_moves`` (default 10^8; 0: unbounded) caps one worm.'''

    DEVICE_KIND = 'villain'

    def __init__(self, S, *, device=None, max_moves=WORM_MAX_MOVES):
        if not _is_villain(S):
            raise ValueError('Need a Villain action')
        if S.Lattice.D != 2:
            raise NotImplementedError('ClassicWorm is only implemented for D=2')
        self.Action = S
        self.rng = np.random.default_rng()
        self.worm_lengths = __import__('collections').deque()
        self.plaquette = np.array([+1, +1, -1, -1])  # east, north, west, south (worm.py:68)
        self.device = device
        self.max_moves = int(max_moves)

    def __str__(self):
        return 'ClassicWorm'

    _state = _VillainLocal._state
    __del__ = _VillainLocal.__del__
    _fields = _VillainLocal._fields

    @property
    def Lattice(self):
        return self.Action.Lattice

    def inline_observables(self, steps):
        L = self.Action.Lattice
        return {
            'Vortex_Vortex': Batch(steps, shape=(L.N, L.N)),
            'Worm_Length': Batch(steps, shape=(), dtype=float),
        }

    def _run_on(self, ctx, h, count):
        """`count` worms on the device-resident (phi, n); returns (last histogram, last length)."""
        N = self.Action.Lattice.N
        hist = np.zeros((N, N), dtype=np.int64)
        lengths = np.zeros(count, dtype=np.int64)
        W = self.Action.W
        r = rng_from_numpy(self.rng)
        ctx.check(_native.lib().sv_villain_worm_run(h, float(self.Action.kappa), 1 if W == 1 else 0, int(count),
                                                    self.max_moves, ctypes.byref(r), _native.ptr(hist),
                                                    _native.ptr(lengths)), 'sv_villain_worm_run')
        rng_to_numpy(r, self.rng)
        self.worm_lengths.extend(np.int64(x) for x in lengths)
        return hist, lengths[-1]

    def _inline_dict(self, out):
        return {'Vortex_Vortex': out[0], 'Worm_Length': out[1]}

    def _steps(self, cfg, count):
        phi, n = self._fields(cfg)
        ctx, N, h = self._state()
        L = _native.lib()
        ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_upload')
        hist, wl = self._run_on(ctx, h, count)
        ctx.check(L.sv_villain_download(h, _native.ptr(phi), _native.ptr(n)), 'sv_villain_download')
        return cfg | {'n': wrap_like(cfg['n'], n, 1, self.Action.Lattice), 'Vortex_Vortex': hist, 'Worm_Length': wl}

    def step(self, cfg):
        return self._steps(cfg, 1)

    def report(self):
        return _worm_report(self.worm_lengths)


Worm = ClassicWorm


def Hammer(S, worms=1, *, worm=True):
    r'''The reference's Villain Hammer (supervillain/generator/villain/__init__.py:11-64):
    Sequentially(Site, Link, Exact, Cohomology, Worm), LinkUpdate omitted at W = infinity.  As in the reference
    the worm is included whenever D == 2, whatever `worms` is, and wrapped in KeepEvery(worms, ...) when
    worms > 1; for D != 2 it is omitted.  ``worm=False`` (not a reference argument) builds the worm-free
    program.'''
    from supervillain_amd.generator.combining import KeepEvery, Sequentially
    tail = ()
    if worm and S.Lattice.D == 2:
        W = ClassicWorm(S)
        tail = (KeepEvery(worms, W) if worms > 1 else W,)
    if S.W < float('inf'):
        return Sequentially((SiteUpdate(S), LinkUpdate(S), ExactUpdate(S), CohomologyUpdate(S)) + tail)
    return Sequentially((SiteUpdate(S), ExactUpdate(S), CohomologyUpdate(S)) + tail)
