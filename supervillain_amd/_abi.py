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


class SvStats(ctypes.Structure):
    _fields_ = [
        ('accepted', ctypes.c_int64),
        ('proposed', ctypes.c_int64),
        ('acceptance_sum', ctypes.c_double),
        ('rejections', ctypes.c_int64),
    ]


def rng_from_numpy(gen):
    """Snapshot a NumPy Generator(PCG64) into an SvRng."""
    st = gen.bit_generator.state
    if st.get('bit_generator') != 'PCG64':
        raise TypeError(f"the device generators replay NumPy's PCG64 stream; got {st.get('bit_generator')}")
    s, inc = int(st['state']['state']), int(st['state']['inc'])
    return SvRng(s >> 64, s & _M64, inc >> 64, inc & _M64, int(st['has_uint32']), int(st['uinteger']) & 0xFFFFFFFF)


def rng_to_numpy(r, gen):
    """Write an SvRng back into the NumPy Generator, so host-side draws continue the same stream."""
    st = gen.bit_generator.state
    st['state'] = {'state': (int(r.state_hi) << 64) | int(r.state_lo), 'inc': (int(r.inc_hi) << 64) | int(r.inc_lo)}
    st['has_uint32'] = int(r.has_uint32)
    st['uinteger'] = int(r.uinteger)
    gen.bit_generator.state = st
