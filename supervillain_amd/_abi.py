"""ctypes mirrors of the C-ABI structs declared in include/supervillain_amd.h.

The generator's random state stays a NumPy ``np.random.Generator`` (PCG64), exactly as in the
reference (e.g. supervillain/generator/villain/neighborhood.py:50 ``self.rng = np.random.default_rng()``);
it crosses the boundary as its raw 128-bit state, increment and the 32-bit half-word buffer that
NumPy's bounded-integer sampler keeps in the bit generator (``has_uint32``/``uinteger``).
"""
import ctypes

import numpy as np

_M64 = (1 << 64) - 1


class SvRng(ctypes.Structure):
    _fields_ = [
        ('state_hi', ctypes.c_uint64),
        ('state_lo', ctypes.c_uint64),
        ('inc_hi', ctypes.c_uint64),
        ('inc_lo', ctypes.c_uint64),
        ('has_uint32', ctypes.c_int32),
        ('uinteger', ctypes.c_uint32),
    ]


class SvPhilox(ctypes.Structure):
    """sv_philox: the optional counter-based mode's key, sweeps done, and a test-only rejection threshold."""
    _fields_ = [('key', ctypes.c_uint64), ('counter', ctypes.c_uint64), ('test_threshold', ctypes.c_uint32)]


class SvStats(ctypes.Structure):
    _fields_ = [
        ('accepted', ctypes.c_int64),
        ('proposed', ctypes.c_int64),
        ('acceptance_sum', ctypes.c_double),
        ('rejections', ctypes.c_int64),
    ]


class SvMT19937(ctypes.Structure):
    """sv_mt19937: NumPy's legacy global RandomState (MT19937) key and position (include/supervillain_amd.h)."""
    _fields_ = [('key', ctypes.c_uint32 * 624), ('pos', ctypes.c_int32)]


def legacy_state_get():
    """The legacy global RandomState (np.random.seed / np.random.permutation) as an SvMT19937, plus the parts of
    np.random.get_state() a permutation does not touch (has_gauss, cached_gaussian)."""
    name, key, pos, has_gauss, gauss = np.random.get_state(legacy=True)
    if name != 'MT19937':
        raise ValueError(f'unexpected legacy bit generator {name}')
    mt = SvMT19937()
    ctypes.memmove(mt.key, np.ascontiguousarray(key, dtype=np.uint32).ctypes.data, 624 * 4)
    mt.pos = int(pos)
    return mt, (has_gauss, gauss)


def legacy_state_set(mt, rest):
    """Write an SvMT19937 back into NumPy's legacy global RandomState."""
    key = np.frombuffer(bytes(mt.key), dtype=np.uint32).copy()
    np.random.set_state(('MT19937', key, int(mt.pos), rest[0], rest[1]))


class _PCG64State(ctypes.Structure):
    """NumPy's pcg64_state (numpy/random/src/pcg64/pcg64.h): the PCG state pointer and the half-word buffer."""
    _fields_ = [('pcg', ctypes.c_void_p), ('has_uint32', ctypes.c_int), ('uinteger', ctypes.c_uint32)]


_RAW_OK = None  # the raw layout is checked against the state dict once per process


def _raw(gen):
    """(pcg64_state, uint64[4] = state lo, hi, inc lo, hi) views of a PCG64 bit generator, or None when this
    NumPy build's layout differs (then the public state dict is used)."""
    global _RAW_OK
    bg = gen.bit_generator
    if _RAW_OK is False or type(bg).__name__ != 'PCG64':
        return None
    try:
        st = _PCG64State.from_address(bg.ctypes.state_address)
        w = (ctypes.c_uint64 * 4).from_address(st.pcg)
    except Exception:
        _RAW_OK = False
        return None
    if _RAW_OK is None:
        d = bg.state
        _RAW_OK = (d['state']['state'] == (w[1] << 64 | w[0]) and d['state']['inc'] == (w[3] << 64 | w[2])
                   and d['has_uint32'] == st.has_uint32 and d['uinteger'] == st.uinteger)
        if not _RAW_OK:
            return None
    return st, w


def rng_from_numpy(gen):
    """Snapshot a NumPy Generator(PCG64) into an SvRng."""
    raw = _raw(gen)
    if raw is not None:
        st, w = raw
        return SvRng(w[1], w[0], w[3], w[2], st.has_uint32, st.uinteger)
    st = gen.bit_generator.state
    if st.get('bit_generator') != 'PCG64':
        raise TypeError(f"the device generators replay NumPy's PCG64 stream; got {st.get('bit_generator')}")
    s, inc = int(st['state']['state']), int(st['state']['inc'])
    return SvRng(s >> 64, s & _M64, inc >> 64, inc & _M64, int(st['has_uint32']), int(st['uinteger']) & 0xFFFFFFFF)


def rng_to_numpy(r, gen):
    """Write an SvRng back into the NumPy Generator, so host-side draws continue the same stream."""
    raw = _raw(gen)
    if raw is not None:
        st, w = raw
        w[0], w[1], w[2], w[3] = r.state_lo, r.state_hi, r.inc_lo, r.inc_hi
        st.has_uint32, st.uinteger = r.has_uint32, r.uinteger
        return
    st = gen.bit_generator.state
    st['state'] = {'state': (int(r.state_hi) << 64) | int(r.state_lo), 'inc': (int(r.inc_hi) << 64) | int(r.inc_lo)}
    st['has_uint32'] = int(r.has_uint32)
    st['uinteger'] = int(r.uinteger)
    gen.bit_generator.state = st


def rngs_from_numpy(gens):
    """SvRng array of many Generators: one C call over their raw states when the layout checks out."""
    from supervillain_amd import _native
    R = len(gens)
    out = (SvRng * R)()
    if R and _raw(gens[0]) is not None and all(type(g.bit_generator).__name__ == 'PCG64' for g in gens):
        addrs = (ctypes.c_void_p * R)(*[g.bit_generator.ctypes.state_address for g in gens])
        if _native.lib().sv_rng_gather(addrs, R, out) == 0:
            return out, addrs
    for i, g in enumerate(gens):
        out[i] = rng_from_numpy(g)
    return out, None


def rngs_to_numpy(arr, gens, addrs=None):
    """Write an SvRng array back into its Generators (the addresses from rngs_from_numpy when available)."""
    from supervillain_amd import _native
    if addrs is not None and _native.lib().sv_rng_scatter(arr, len(gens), addrs) == 0:
        return
    for x, g in zip(arr, gens):
        rng_to_numpy(x, g)
