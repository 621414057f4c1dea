"""Test-tooling shim that imports the READ-ONLY reference (/root/reference) in THIS container.

Container-only: never imported by the product, never shipped to the GPU box (the reference is
absent there).  Used only by tools/make_golden.py to capture golden vectors.

Why a shim: the reference declares python>=3.14 and depends on numba + h5py,
neither of which is installed here.  The shim
  1. stubs `numba` (njit -> identity, prange -> range, jitclass -> identity),
  2. stubs `h5py` (names only; h5 I/O is out of scope),
  3. rewrites PEP-646 star-subscripts `x[a, *b]` -> `x[(a, *b)]` at import time (semantically
     identical; 3.10 cannot parse the former),
  4. routes the lattice operators to the reference's own pure-NumPy oracles in
     supervillain/lattice/reference.py, which test/test_lattice_kernels.py pins bit-identical to the
     numba kernels.
"""
import importlib.abc
import importlib.machinery
import importlib.util
import re
import sys
import types

REFERENCE = '/root/reference'
_STAR = re.compile(r'(\w|\])\[([^\[\]()\n]+?), \*(\w+)\]')


def _stub_numba():
    nb = types.ModuleType('numba')

    def njit(*args, **kw):
        if args and callable(args[0]) and not kw:
            return args[0]
        return lambda f: f

    nb.njit = njit
    nb.jit = njit
    nb.prange = range
    class _T:
        def __getitem__(self, k):
            return self

        def __call__(self, *a, **k):
            return self

    for t in ('int64', 'float64', 'int32', 'boolean', 'uint64', 'complex128', 'int8'):
        setattr(nb, t, _T())
    exp = types.ModuleType('numba.experimental')
    exp.jitclass = lambda *a, **k: (a[0] if a and isinstance(a[0], type) else (lambda c: c))
    nb.experimental = exp
    typ = types.ModuleType('numba.types')
    nb.types = typ
    sys.modules['numba'] = nb
    sys.modules['numba.experimental'] = exp
    sys.modules['numba.types'] = typ


def _stub_h5py():
    h5 = types.ModuleType('h5py')

    class _Any:
        def __init__(self, *a, **k):
            raise RuntimeError('h5py is stubbed in the golden-vector shim')

    h5.File = h5.Group = h5.Dataset = _Any
    h5.special_dtype = lambda **k: None
    h5.string_dtype = lambda *a, **k: None
    sys.modules['h5py'] = h5


class _RewritingLoader(importlib.machinery.SourceFileLoader):
    def get_data(self, path):
        data = super().get_data(path)
        if path.endswith('.py'):
            text = data.decode('utf-8')
            prev = None
            while prev != text:
                prev = text
                text = _STAR.sub(lambda m: f'{m.group(1)}[({m.group(2)}, *{m.group(3)})]', text)
            data = text.encode('utf-8')
        return data

    def path_stats(self, path):  # defeat bytecode caching of the rewritten source
        raise OSError


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path, target=None):
        if not (name == 'supervillain' or name.startswith('supervillain.')):
            return None
        spec = importlib.machinery.PathFinder.find_spec(name, path or [REFERENCE])
        if spec is None or spec.origin is None or not spec.origin.endswith('.py'):
            return spec
        spec.loader = _RewritingLoader(name, spec.origin)
        return spec


def load():
    """Import and return the reference `supervillain` package through the shim."""
    if 'supervillain' in sys.modules:
        return sys.modules['supervillain']
    sys.dont_write_bytecode = True
    _stub_numba()
    _stub_h5py()
    sys.meta_path.insert(0, _Finder())
    import supervillain
    from supervillain.lattice import compact, reference
    ops = {'d': reference.reference_d, 'delta': reference.reference_delta,
           'face_sum': reference.reference_face_sum, 'coface_sum': reference.reference_coface_sum}

    def _apply_operator(kernels, op, f, out_degree):
        return ops[op](f)

    compact._apply_operator = _apply_operator
    return supervillain
