"""The C-ABI library loads and exports every symbol include/supervillain_amd.h declares (CPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'supervillain_amd.h')


def declared():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(sv_[a-z0-9_]+)\s*\(', text)))


@pytest.fixture(scope='module')
def lib():
    from supervillain_amd import _native
    return _native.lib()


def test_header_declares_the_boundary():
    names = declared()
    for must in ('sv_villain_neighborhood', 'sv_worldline_coexact', 'sv_worldline_plaquette', 'sv_ctx_create'):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from supervillain_amd import _native
    assert sorted(_native.EXPORTED) == declared()


def test_structs_match_header_sizes():
    from supervillain_amd._abi import SvRng, SvStats
    assert ctypes.sizeof(SvRng) == 40
    assert ctypes.sizeof(SvStats) == 32


def test_no_device_fails_loudly(lib):
    from supervillain_amd import _native
    if lib.sv_device_count() > 0:
        pytest.skip('a GPU is present')
    with pytest.raises(_native.NativeError):
        _native.Context(0)
