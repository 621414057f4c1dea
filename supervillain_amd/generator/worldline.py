"""Worldline hot-path generators on the MI355X.

CoexactUpdate   supervillain/generator/worldline/coexact.py:12-194
PlaquetteUpdate supervillain/generator/worldline/plaquette.py:9-113

Same constructors, attributes, `step` contracts and `report()` texts as the reference; the sweeps
run in libsvhip.so (include/supervillain_amd.h) replaying `self.rng`'s NumPy PCG64 stream.
"""
import ctypes

import numpy as np

from supervillain_amd import _native
from supervillain_amd._abi import legacy_state_get, legacy_state_set
from supervillain_amd.generator._common import DeviceState, rng_from_numpy, rng_to_numpy, wrap_like
from supervillain_amd.generator.generator import Generator
from supervillain_amd.replicas import WORM_MAX_MOVES


def _is_worldline(action):
    return type(action).__name__ == 'Worldline' and hasattr(action, '_W') and hasattr(action, 'Lattice')


class _WorldlineDevice(DeviceState):
    def _state(self):
        L = self.Action.Lattice
        if L.D != 2:
            raise NotImplementedError(f'the MI355X {self} is implemented for D=2 lattices')
        v_float = not (self.Action.W < float('inf'))
        dev = self.__dict__.get('_dev')
        if dev is None or dev[1] != (L.N, v_float):
            ctx = self._device_context()
            h = ctypes.c_void_p()
            ctx.check(_native.lib().sv_worldline_create(ctx.handle, L.N, int(v_float), ctypes.byref(h)),
                      'sv_worldline_create')
            dev = (ctx, (L.N, v_float), h)
            self._dev = dev
        return dev

    def __del__(self):
        dev = self.__dict__.get('_dev')
        if dev is not None and _native._LIB is not None:
            self._dev = None
            _native.destroy(_native._LIB.sv_worldline_destroy, dev[2], 'sv_worldline_destroy (' + type(self).__name__ + ')', dev[0], in_del=True)

    def _fields(self, cfg):
        N = self.Action.Lattice.N
        m = np.array(cfg['m'], dtype=np.int64, order='C', copy=True).reshape(2, N, N)
        v_float = not (self.Action.W < float('inf'))
        v = np.array(cfg['v'], dtype=np.float64 if v_float else np.int64, order='C', copy=True).reshape(1, N, N)
        return m, v


class CoexactUpdate(_WorldlineDevice, Generator):
    r'''Changes m by delta t with t = ±1..±interval_t on one plaquette colour at a time (coexact.py:12-31).'''

    def __init__(self, action, interval_t=1, *, device=None):
        if not _is_worldline(action):
            raise ValueError('Need a Worldline action')
        self.Action = action
        self.Lattice = action.Lattice
        self.kappa = action.kappa
        self.interval_t = interval_t
        self.ts = tuple(range(-interval_t, 0)) + tuple(range(1, interval_t + 1))
        self.rng = np.random.default_rng()
        self.accepted = 0
        self.proposed = 0
        self.acceptance = 0.
        self.sweeps = 0
        self.device = device

    def __str__(self):
        return 'SiteUpdate'  # sic: the reference's CoexactUpdate.__str__ (coexact.py:50-51)

    DEVICE_KIND = 'worldline'

    def _run_on(self, ctx, h, sweeps):
        L = _native.lib()
        st = _native.stats_array(sweeps)
        r = rng_from_numpy(self.rng)
        ctx.check(L.sv_worldline_coexact_run(h, float(self.kappa), float(self.Action._W), int(self.interval_t),
                                             sweeps, ctypes.byref(r), st), 'sv_worldline_coexact_run')
        rng_to_numpy(r, self.rng)
        P = self.Lattice.cells_of_degree[2]

        def fold():
            for k in range(sweeps):  # coexact.py:122-124
                self.sweeps += 1
                self.proposed += P
                self.acceptance += st[k].acceptance_sum / P
                self.accepted += int(st[k].accepted)
        ctx.fold_later(fold)
        return None

    def _advance(self, cfg, sweeps):
        ctx, _, h = self._state()
        m, v = self._fields(cfg)
        L = _native.lib()
        ctx.check(L.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_upload')
        self._run_on(ctx, h, sweeps)
        ctx.check(L.sv_worldline_download(h, _native.ptr(m), None), 'sv_worldline_download')
        return cfg | {'m': wrap_like(cfg['m'], m, 1, self.Lattice)}

    def step(self, cfg):
        return self._advance(cfg, 1)

    def _steps(self, cfg, count):
        return self._advance(cfg, count)

    def report(self):
        return (
            f'There were {self.accepted} coexact proposals accepted of {self.proposed} proposed updates.'
            + '\n' +
            f'    {self.accepted/self.proposed:.6f} acceptance rate'
            + '\n' +
            f'    {self.acceptance / self.sweeps:.6f} average Metropolis acceptance probability.'
        )


class PlaquetteUpdate(_WorldlineDevice, Generator):
    r'''Single-plaquette Metropolis on the 4 boundary links of m and on v (plaquette.py:9-22).

    mode='reference' (default) keeps the reference's chain: every sweep visits the plaquettes in the
    order np.random.permutation(L.coordinates) draws from NumPy's global RandomState, exactly as
    plaquette.py:63 does, and the device processes them in dependency rounds that reproduce the
    sequential loop bit-for-bit.  mode='checkerboard' is the GPU-native variant: colour
    passes, no global-RandomState draw, a different but equally valid chain.
    '''

    def __init__(self, action, *, mode='reference', device=None):
        if not _is_worldline(action):
            raise ValueError('The PlaquetteUpdate requires the Worldline action.')
        if mode not in ('reference', 'checkerboard'):
            raise ValueError("mode must be 'reference' or 'checkerboard'")
        self.Action = action
        self.accepted = 0
        self.proposed = 0
        self.rng = np.random.default_rng()
        self.acceptance = 0.
        self.mode = mode
        self.device = device

    def __str__(self):
        return 'PlaquetteUpdate'

    DEVICE_KIND = 'worldline'

    def _run_on(self, ctx, h, sweeps):
        Lib = _native.lib()
        L = self.Action.Lattice
        r = rng_from_numpy(self.rng)
        kappa, W = float(self.Action.kappa), float(self.Action._W)
        if self.mode == 'reference':
            # plaquette.py:63's np.random.permutation(L.coordinates) -- NumPy's legacy global RandomState, whose
            # row-major coordinates make the visit order the shuffled index array itself -- drawn natively from the
            # same MT19937 state (sv_mt19937_permutation), which advances exactly as NumPy's would
            mt, rest = legacy_state_get()
            st = _native.stats_array(sweeps)
            ctx.check(Lib.sv_worldline_plaquette_reference_run(h, kappa, W, sweeps, ctypes.byref(mt), ctypes.byref(r), st),
                      'sv_worldline_plaquette_reference_run')
            legacy_state_set(mt, rest)
            stats = lambda: [(int(st[k].accepted), st[k].acceptance_sum) for k in range(sweeps)]  # noqa: E731
        else:
            st = _native.stats_array(sweeps)
            ctx.check(Lib.sv_worldline_plaquette_checkerboard_run(h, kappa, W, sweeps, ctypes.byref(r), st),
                      'sv_worldline_plaquette_checkerboard_run')
            stats = lambda: [(int(st[k].accepted), st[k].acceptance_sum) for k in range(sweeps)]  # noqa: E731
        rng_to_numpy(r, self.rng)
        P = L.sites * len(L.components[2])

        def fold():
            for acc, psum in stats():  # plaquette.py:73, 101-103
                self.acceptance += psum
                self.accepted += acc
                self.proposed += P
        ctx.fold_later(fold)
        return None

    def _advance(self, cfg, sweeps):
        ctx, _, h = self._state()
        m, v = self._fields(cfg)
        Lib = _native.lib()
        L = self.Action.Lattice
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_upload')
        self._run_on(ctx, h, sweeps)
        ctx.check(Lib.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_download')
        return cfg | {'m': wrap_like(cfg['m'], m, 1, L), 'v': wrap_like(cfg['v'], v, 2, L)}

    def step(self, cfg):
        return self._advance(cfg, 1)

    def _steps(self, cfg, count):
        return self._advance(cfg, count)

    def report(self):
        return (
            f'There were {self.accepted} single-plaquette proposals accepted of {self.proposed} proposed updates.'
            + '\n' +
            f'    {self.accepted/self.proposed:.6f} acceptance rate'
            + '\n' +
            f'    {self.acceptance / self.proposed :.6f} average Metropolis acceptance probability.'
        )


# ------------------------------------------------------------------------------------------------
# The rest of the Worldline Hammer: VortexUpdate (v only) and WrappingUpdate (m on whole
# torus cycles).  Same constructors, attributes, `step` contracts and `report()` text as the reference.

class _WorldlineLocal(_WorldlineDevice, Generator):
    NAME = None
    NOUN = None
    FIELD = None  # 'm' or 'v': what the step returns

    def _init_common(self, action, device, message):
        if not _is_worldline(action):
            raise ValueError(message)
        self.Action = action
        self.accepted = 0
        self.proposed = 0
        self.acceptance = 0.
        self.sweeps = 0
        self.rng = np.random.default_rng()
        self.device = device

    def __str__(self):
        return self.NAME

    DEVICE_KIND = 'worldline'

    def _run_on(self, ctx, h, sweeps):
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

    def _advance(self, cfg, sweeps):
        ctx, _, h = self._state()
        m, v = self._fields(cfg)
        L = _native.lib()
        ctx.check(L.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_upload')
        self._run_on(ctx, h, sweeps)
        ctx.check(L.sv_worldline_download(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_download')
        Lat = self.Action.Lattice
        if self.FIELD == 'm':
            return cfg | {'m': wrap_like(cfg['m'], m, 1, Lat)}
        return cfg | {'v': wrap_like(cfg['v'], v, 2, Lat)}

    def step(self, cfg):
        return self._advance(cfg, 1)

    def _steps(self, cfg, count):
        return self._advance(cfg, count)

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


class VortexUpdate(_WorldlineLocal):
    r'''Checkerboard Metropolis update of v alone, m untouched (supervillain/generator/worldline/vortex.py:12-190):
    Δv ~ {-interval_v..-1, 1..interval_v} (finite W) or uniform(-interval_v, interval_v) (W = ∞).'''

    NAME = 'VortexUpdate'
    NOUN = 'vortex'
    FIELD = 'v'

    def __init__(self, action, interval_v=1, *, device=None):
        self._init_common(action, device, 'Need a Worldline action')
        self.interval_v = interval_v
        self.vs = tuple(v for v in range(-interval_v, 0)) + tuple(v for v in range(1, interval_v + 1))

    def _proposals(self):
        return self.Action.Lattice.cells_of_degree[2]

    def _run(self, L, h, sweeps, r, st):
        return L.sv_worldline_vortex_run(h, float(self.Action.kappa), float(self.Action._W), int(self.interval_v),
                                         sweeps, ctypes.byref(r), st)


class WrappingUpdate(_WorldlineLocal):
    r'''Coordinated changes of m on whole torus cycles, Δm ~ {-interval_w..-1, 1..interval_w} on every link of the
    cycle (supervillain/generator/worldline/wrapping.py:9-98).'''

    NAME = 'WrappingUpdate'
    NOUN = 'single-wrapping'
    FIELD = 'm'

    def __init__(self, action, interval_w=1, *, device=None):
        self._init_common(action, device, 'The WrappingUpdate requires the Worldline action.')
        self.interval_w = interval_w
        self.w = tuple(h for h in range(-interval_w, 0)) + tuple(h for h in range(1, interval_w + 1))

    def _proposals(self):
        L = self.Action.Lattice
        return L.D * L.N ** (L.D - 1)  # n_cycles, wrapping.py:86

    def _run(self, L, h, sweeps, r, st):
        return L.sv_worldline_wrapping_run(h, float(self.Action.kappa), float(self.Action._W), int(self.interval_w),
                                           sweeps, ctypes.byref(r), st)


class ClassicWorm(_WorldlineDevice, Generator):
    r'''The Prokof'ev-Svistunov worm on the worldline links (supervillain/generator/worldline/worm.py:97-193):
    head and tail on sites, the head crosses links changing m by ±1; the displacement histogram is the inline
    ``Spin_Spin`` measurement.  One chain per GPU lane (``sv_worldline_worm_run``); batches of chains use
    :func:`supervillain_amd.replicas.worldline_worms`.  ``max_moves`` (default 10^8; 0: unbounded) caps one worm.'''

    DEVICE_KIND = 'worldline'

    def __init__(self, S, *, device=None, max_moves=WORM_MAX_MOVES):
        if not _is_worldline(S):
            raise ValueError('The classic worm algorithm update requires the Worldline action.')
        self.Action = S
        self.rng = np.random.default_rng()
        self.worm_lengths = __import__('collections').deque()
        D = S.Lattice.D
        self.divergence = np.array([+1] * D + [-1] * D, dtype=int)  # worm.py:135
        self.device = device
        self.max_moves = int(max_moves)

    def __str__(self):
        return 'ClassicWorm'

    def inline_observables(self, steps):
        from supervillain_amd.batch import Batch
        L = self.Action.Lattice
        return {
            'Spin_Spin': Batch(steps, shape=L.dims),
            'Worm_Length': Batch(steps, shape=(), dtype=float),
        }

    def _run_on(self, ctx, h, count):
        N = self.Action.Lattice.N
        hist = np.zeros((N, N), dtype=np.int64)
        lengths = np.zeros(count, dtype=np.int64)
        r = rng_from_numpy(self.rng)
        ctx.check(_native.lib().sv_worldline_worm_run(h, float(self.Action.kappa), float(self.Action._W), int(count),
                                                      self.max_moves, ctypes.byref(r), _native.ptr(hist),
                                                      _native.ptr(lengths)), 'sv_worldline_worm_run')
        rng_to_numpy(r, self.rng)
        self.worm_lengths.extend(int(x) for x in lengths)
        return hist, int(lengths[-1])

    def _inline_dict(self, out):
        return {'Spin_Spin': out[0], 'Worm_Length': out[1]}

    def _steps(self, cfg, count):
        ctx, _, h = self._state()
        m, v = self._fields(cfg)
        L = _native.lib()
        ctx.check(L.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_upload')
        hist, wl = self._run_on(ctx, h, count)
        ctx.check(L.sv_worldline_download(h, _native.ptr(m), None), 'sv_worldline_download')
        return cfg | {'m': wrap_like(cfg['m'], m, 1, self.Action.Lattice), 'Spin_Spin': hist, 'Worm_Length': wl}

    def step(self, cfg):
        return self._steps(cfg, 1)

    def report(self):
        l = np.array(self.worm_lengths)
        return f'There were {len(l)} worms.\nWorms lengths:\n    mean {l.mean()}\n    std  {l.std()}\n    max  {max(l)}'


Worm = ClassicWorm


def Hammer(S, worms=1, *, worm=True):
    r'''The reference's Worldline Hammer (supervillain/generator/worldline/__init__.py:10-41):
    Sequentially(Vortex, Coexact, Wrapping, Worm), the worm always included, whatever `worms` is, and wrapped in
    KeepEvery(worms, ...) when worms > 1.  ``worm=False`` (not a reference argument) builds the worm-free
    program.'''
    from supervillain_amd.generator.combining import KeepEvery, Sequentially
    tail = ()
    if worm:
        W = ClassicWorm(S)
        tail = (KeepEvery(worms, W) if worms > 1 else W,)
    return Sequentially((VortexUpdate(S), CoexactUpdate(S), WrappingUpdate(S)) + tail)
