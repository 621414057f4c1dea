"""Host-side lattice and p-form types the generators exchange with their callers.

Mirrors the parts of supervillain.lattice that the hot path's callers touch
(supervillain/lattice/compact.py:60-261 Lattice, :665-890 Form, :973-1037 d/delta,
two_dimensional.py:9-60 Lattice2D): the storage layout (C(D,p), N, ..., N), the checkerboard
colouring (compact.py:191-239) and the exterior-derivative operators used by the actions'
constraint checks.  These run on the host in NumPy; the sweeps themselves run in libsvhip.so.
"""
from functools import cached_property
from itertools import combinations
from math import comb

import numpy as np


def _fft_coordinates(n):
    """FFT-convention coordinates of a periodic direction: 0..n//2 then -(n-1)//2..-1 (lattice/__init__.py:4-9)."""
    c = np.arange(n)
    return np.where(c <= n // 2, c, c - n)


class Lattice:
    """A D-dimensional periodic hypercubic lattice with N sites per direction (compact.py:60)."""

    def __init__(self, D, N):
        self.D = int(D)
        self.N = int(N)
        self.components = {p: list(combinations(range(self.D), p)) for p in range(self.D + 1)}
        self.comp_index = {p: {c: i for i, c in enumerate(self.components[p])} for p in range(self.D + 1)}

    def __repr__(self):
        return f'Lattice(D={self.D}, N={self.N})'

    @cached_property
    def sites(self):
        return self.N ** self.D

    @cached_property
    def dims(self):
        return (self.N,) * self.D

    @property
    def dim(self):
        return self.D

    @cached_property
    def links(self):
        return self.D * self.sites

    @cached_property
    def cells_of_degree(self):
        return {p: comb(self.D, p) * self.sites for p in range(self.D + 1)}

    @cached_property
    def _coord_1d(self):
        return _fft_coordinates(self.N)

    @cached_property
    def coords(self):
        """FFT-convention coordinate of every site, shape (D, N, ..., N)."""
        return np.stack(np.meshgrid(*([self._coord_1d] * self.D), indexing='ij'), axis=0)

    @cached_property
    def coordinates(self):
        """(sites, D) array of FFT-convention coordinates in row-major site order."""
        return np.stack([c.ravel() for c in np.meshgrid(*([self._coord_1d] * self.D), indexing='ij')], axis=1)

    def mod(self, x):
        return self._coord_1d[np.mod(np.asarray(x), self.N)]

    @cached_property
    def checkerboarding(self):
        """Site colours with no same-colour nearest neighbours (compact.py:191-239).

        Even N: the two parities of the coordinate sum.  Odd N: 2^max(D,2) colours, each a pair of
        opposite hyperoctants (on FFT coordinates) split by parity.  Each colour is an np.where
        tuple, so its sites come in row-major order -- the order the generators draw in."""
        coords = self.coords
        parity = np.mod(coords.sum(axis=0), 2)
        if self.N % 2 == 0:
            return tuple(np.where(parity == c) for c in (0, 1))
        colours = []
        for b in range(1 << max(self.D - 1, 1)):
            if self.D == 1:
                pair = coords[0] >= 0 if b == 0 else coords[0] < 0
            else:
                pos = coords[0] >= 0
                neg = coords[0] < 0
                for k in range(1, self.D):
                    flip = (b >> (k - 1)) & 1
                    pos = pos & ((coords[k] < 0) if flip else (coords[k] >= 0))
                    neg = neg & ((coords[k] >= 0) if flip else (coords[k] < 0))
                pair = pos | neg
            for c in (0, 1):
                colours.append(np.where(pair & (parity == c)))
        return tuple(colours)

    def zeros(self, p, dtype=float):
        shape = (comb(self.D, p),) + self.dims
        return Form(np.zeros(shape, dtype=dtype), degree=p, lattice=self)

    form = zeros


class Lattice2D(Lattice):
    """A two-dimensional square lattice (two_dimensional.py:9-60)."""

    def __init__(self, n):
        super().__init__(D=2, N=n)

    @property
    def plaquettes(self):
        return self.cells_of_degree[2]

    @property
    def nt(self):
        return self.N

    @property
    def nx(self):
        return self.N

    @property
    def t(self):
        return self._coord_1d

    @property
    def x(self):
        return self._coord_1d


class Form(np.ndarray):
    """A p-form: an ndarray of shape (C(D,p), N, ..., N) carrying its degree and lattice (compact.py:665).

    Elementwise ufuncs on Forms of one degree return a Form; anything else is a plain ndarray."""

    __batch_tag__ = 'Form'

    @classmethod
    def spatial_shape(cls, *, degree, lattice):
        return (comb(lattice.D, degree),) + lattice.dims

    def __new__(cls, input_array, *, degree, lattice, dtype=None):
        obj = np.asarray(input_array, dtype=dtype).view(cls)
        obj.degree = degree
        obj.lattice = lattice
        return obj

    def __array_finalize__(self, obj):
        if obj is None:
            return
        self.degree = getattr(obj, 'degree', None)
        self.lattice = getattr(obj, 'lattice', None)

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        forms = [x for x in inputs if isinstance(x, Form)]
        degrees = {f.degree for f in forms}
        raw = tuple(np.asarray(x) for x in inputs)
        if 'out' in kwargs:
            kwargs['out'] = tuple(np.asarray(o) for o in kwargs['out'])
        result = getattr(ufunc, method)(*raw, **kwargs)
        if len(degrees) == 1 and isinstance(result, np.ndarray) and result.shape == forms[0].shape:
            return Form(result, degree=forms[0].degree, lattice=forms[0].lattice)
        return result

    def face_sum(self):
        if self.degree == 0:
            return 0
        return _unsigned(self, down=True)

    def coface_sum(self):
        if self.degree == self.lattice.D:
            return 0
        return _unsigned(self, down=False)


def _tables(lat, op, p):
    """(out, in, axis, sign) incidence rows in the reference's row order (compact.py:143-174)."""
    rows = []
    if op in ('d', 'coface_sum'):
        for out_comp in lat.components[p + 1]:
            for j, k in enumerate(out_comp):
                in_comp = tuple(a for a in out_comp if a != k)
                rows.append((lat.comp_index[p + 1][out_comp], lat.comp_index[p][in_comp], k,
                             (-1) ** j if op == 'd' else 1))
    else:
        for out_comp in lat.components[p - 1]:
            for e in sorted(set(range(lat.D)) - set(out_comp)):
                j = sum(1 for a in out_comp if a < e)
                in_comp = tuple(sorted(set(out_comp) | {e}))
                rows.append((lat.comp_index[p - 1][out_comp], lat.comp_index[p][in_comp], e,
                             (-1) ** j if op == 'delta' else 1))
    return rows


def d(f):
    """Exterior derivative (compact.py:973): (df)_O[x] = sum_j (-1)^j (f[x+e_oj] - f[x]), dtype preserved."""
    lat, p = f.lattice, f.degree
    if p == lat.D:
        return 0
    out = lat.zeros(p + 1, dtype=f.dtype)
    A = np.asarray(f)
    for o, i, k, s in _tables(lat, 'd', p):
        out[o] += s * (np.roll(A[i], -1, axis=k) - A[i])
    return out


def delta(f):
    """Codifferential (compact.py:1008): (delta f)_M[x] = -sum (-1)^j (f[x] - f[x-e]), dtype preserved."""
    lat, p = f.lattice, f.degree
    if p == 0:
        return 0
    out = lat.zeros(p - 1, dtype=f.dtype)
    A = np.asarray(f)
    for o, i, e, s in _tables(lat, 'delta', p):
        out[o] -= s * (A[i] - np.roll(A[i], 1, axis=e))
    return out


def _unsigned(f, down):
    lat, p = f.lattice, f.degree
    out = lat.zeros(p - 1 if down else p + 1, dtype=f.dtype)
    A = np.asarray(f)
    for o, i, e, _ in _tables(lat, 'face_sum' if down else 'coface_sum', p):
        out[o] += A[i]
        out[o] += np.roll(A[i], 1 if down else -1, axis=e)
    return out
