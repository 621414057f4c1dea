"""Device-resident Markov chain: Ensemble.generate without a host round trip per step.

The reference's Ensemble.generate (supervillain/ensemble.py:74-98) calls `generator.step(cfg)` once per
configuration; with device generators every step would upload the fields, sweep, and download them again,
and a Sequentially (a Hammer) would do that once per member generator.  Here the whole chain lives in one
device state for the run:

    program = device_program(generator)   # [(leaf generator, sweeps), ...] per emitted configuration
    chain = DeviceChain(action, program)
    chain.upload(seed)
    for i in range(steps):
        obs = chain.advance()              # every leaf runs its sweeps on the resident fields
        chain.emit(phi[i], n[i])           # snapshot on the device, copy to the host on a copy stream
    chain.emit_wait()                      # (the copy of configuration i overlaps the sweeps of i+1)

`device_program` flattens Sequentially (combining.py:9-45) and KeepEvery (combining.py:48-116) into the
leaf generators' own device calls, in the order their `step` methods would run, so the chain -- and every
generator's rng, counters and report -- is exactly the one the host loop produces.  Generators or
compositions it does not know (or a KeepEvery that averages blocked inline observables) return None and
Ensemble.generate keeps the reference's host loop.
"""
import ctypes

import numpy as np

from supervillain_amd import _native
from supervillain_amd.generator.combining import KeepEvery, Sequentially


def device_program(generator):
    """[(leaf, sweeps)] run per emitted configuration, or None if the generator cannot run resident."""
    if isinstance(generator, Sequentially):
        prog = []
        for g in generator.generators:
            p = device_program(g)
            if p is None:
                return None
            prog += p
        return _merge(prog)
    if isinstance(generator, KeepEvery):
        if generator.blocked_inline and generator.inline_observables(1):
            return None  # KeepEvery averages the blocked observables over its stride (combining.py:100-112)
        p = device_program(generator.generator)
        if p is None:
            return None
        return _merge(p * generator.stride)
    if hasattr(generator, '_run_on') and hasattr(generator, 'DEVICE_KIND'):
        return [(generator, 1)]
    return None


def _merge(prog):
    """Consecutive runs of one generator become one device call of several sweeps."""
    out = []
    for g, k in prog:
        if out and out[-1][0] is g:
            out[-1] = (g, out[-1][1] + k)
        else:
            out.append((g, k))
    return out


class DeviceChain:
    """One device-resident (phi, n) or (m, v) state shared by every leaf generator of a program."""

    def __init__(self, action, program):
        kinds = {g.DEVICE_KIND for g, _ in program}
        if len(kinds) != 1:
            raise ValueError('a device program must update one kind of field (Villain or Worldline)')
        self.kind = kinds.pop()
        self.Action = action
        self.program = program
        L = action.Lattice
        if L.D != 2:
            raise NotImplementedError('device-resident chains are implemented for D=2 lattices')
        self.N = L.N
        self.ctx = program[0][0]._device_context()
        self.lib = _native.lib()
        h = ctypes.c_void_p()
        if self.kind == 'villain':
            self.ctx.check(self.lib.sv_villain_create(self.ctx.handle, self.N, ctypes.byref(h)), 'sv_villain_create')
            self.a = np.zeros((1, self.N, self.N))
            self.b = np.zeros((2, self.N, self.N), dtype=np.int64)
            self.names = ('phi', 'n')
        else:
            self.v_float = not (action.W < float('inf'))
            self.ctx.check(self.lib.sv_worldline_create(self.ctx.handle, self.N, int(self.v_float), ctypes.byref(h)),
                           'sv_worldline_create')
            self.a = np.zeros((2, self.N, self.N), dtype=np.int64)
            self.b = np.zeros((1, self.N, self.N), dtype=np.float64 if self.v_float else np.int64)
            self.names = ('m', 'v')
        self.handle = h

    def close(self, _in_del=False):
        if getattr(self, 'handle', None) is not None and _native._LIB is not None:
            h, self.handle = self.handle, None
            fn = _native._LIB.sv_villain_destroy if self.kind == 'villain' else _native._LIB.sv_worldline_destroy
            _native.destroy(fn, h, f'{fn.__name__} (DeviceChain)', self.ctx, _in_del)

    def __del__(self):
        self.close(_in_del=True)

    def upload(self, cfg):
        x, y = self.names
        self.a[...] = np.asarray(cfg[x]).reshape(self.a.shape)
        self.b[...] = np.asarray(cfg[y]).reshape(self.b.shape)
        up = self.lib.sv_villain_upload if self.kind == 'villain' else self.lib.sv_worldline_upload
        self.ctx.check(up(self.handle, _native.ptr(self.a), _native.ptr(self.b)), 'upload')

    def advance(self):
        """Run the program once; returns the inline observables the leaves produced (dict).  The leaves run as one
        deferred step (sv_ctx_set_deferred): members that cannot meet a NumPy Lemire rejection return without a
        synchronization, and one sv_ctx_sync at the end lands every statistic before the counters fold."""
        obs = {}
        self.ctx.begin_deferred()
        try:
            for g, k in self.program:
                out = g._run_on(self.ctx, self.handle, k)
                if out is not None:
                    obs |= g._inline_dict(out)
        finally:
            self.ctx.end_deferred()
        return obs

    def emit(self, a, b):
        """Start copying the resident state into host arrays a, b (returns at once; see sv_villain_emit).  They must
        have this chain's shapes and dtypes, be C-contiguous, and stay untouched until emit_wait()."""
        for h, ref in ((a, self.a), (b, self.b)):
            if h.shape != ref.shape or h.dtype != ref.dtype or not h.flags['C_CONTIGUOUS']:
                raise ValueError(f'emission target {h.shape} {h.dtype} does not match the state {ref.shape} {ref.dtype}')
        em = self.lib.sv_villain_emit if self.kind == 'villain' else self.lib.sv_worldline_emit
        self.ctx.check(em(self.handle, _native.ptr(a), _native.ptr(b)), 'emit')

    def emit_wait(self):
        """Every emission started so far has reached the host."""
        w = self.lib.sv_villain_emit_wait if self.kind == 'villain' else self.lib.sv_worldline_emit_wait
        self.ctx.check(w(self.handle), 'emit_wait')

    def download(self):
        down = self.lib.sv_villain_download if self.kind == 'villain' else self.lib.sv_worldline_download
        self.ctx.check(down(self.handle, _native.ptr(self.a), _native.ptr(self.b)), 'download')
        x, y = self.names
        return {x: self.a, y: self.b}


class _PinnedBlock:
    """Owner of one sv_host_alloc block; freed when the last numpy view of it is gone."""

    def __init__(self, ptr):
        self.ptr = ptr
        self.lib = _native.lib()

    def __del__(self):
        if self.ptr:
            self.lib.sv_host_free(self.ptr)
            self.ptr = None


# below this an emission's copy is short enough that page-locking buys nothing
PIN_MIN_BYTES = 1 << 20


def pinned_empty(shape, dtype):
    """An uninitialised C-contiguous array in page-locked memory the library owns (sv_host_alloc), so that
    emissions into it are DMA copies that overlap the sweeps.  The memory is released when the array and every
    view of it are gone.  Caller arrays are never page-locked in place: numpy storage shares pages with other
    objects, and an overlapping registration can leave the runtime a stale device mapping for them.  Small arrays,
    and a runtime that refuses the allocation, get ordinary memory (copies still land, without the overlap)."""
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    if nbytes < PIN_MIN_BYTES:
        return np.empty(shape, dtype)
    ptr = ctypes.c_void_p()
    if _native.lib().sv_host_alloc(nbytes, ctypes.byref(ptr)) != 0 or not ptr.value:
        return np.empty(shape, dtype)
    raw = (ctypes.c_char * nbytes).from_address(ptr.value)
    raw._owner = _PinnedBlock(ptr.value)
    return np.frombuffer(raw, dtype=dtype).reshape(shape)
