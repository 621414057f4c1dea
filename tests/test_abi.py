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


def _dynamic_symbols(undefined):
    import subprocess
    so = os.path.join(ROOT, 'supervillain_amd', 'libsvhip.so')
    nm = '/opt/rocm/lib/llvm/bin/llvm-nm' if os.path.exists('/opt/rocm/lib/llvm/bin/llvm-nm') else 'nm'
    out = subprocess.run([nm, '-D', '-C', '--undefined-only' if undefined else '--defined-only', so],
                         capture_output=True, text=True, check=True).stdout
    return out


def test_no_caller_memory_is_page_locked():
    """VERDICT r5 next #6, the round-5 fault fix locked in: emission targets are page-locked memory the library
    allocates and owns (sv_host_alloc); nothing registers caller memory in place -- the
    library imports no hipHostRegister, and no Python module names it (or another page-locking call)."""
    und = _dynamic_symbols(True)
    for sym in ('hipHostRegister', 'hipHostUnregister'):
        assert sym not in und, f'libsvhip.so imports {sym}'
    assert 'hipHostMalloc' in und  # (the library's own pinned allocations: sv_host_alloc)
    pkg = os.path.join(ROOT, 'supervillain_amd')
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith('.py'):
                text = open(os.path.join(dirpath, f)).read()
                for bad in ('hipHostRegister', 'cudaHostRegister', 'sv_host_register', 'pin_memory', 'cudart'):
                    assert bad not in text, f'{f} names {bad}'


def test_every_launch_is_sync_checkable():
    """SV_SYNC_CHECK: every kernel launch in csrc/ is followed by SV_LAUNCHED(name, stream), so that
    with SV_SYNC_CHECK=1 a fault names the kernel that caused it; the checker is built into the library."""
    csrc = os.path.join(ROOT, 'supervillain_amd', 'csrc')
    launches = checked = 0
    for f in sorted(os.listdir(csrc)):
        if not f.endswith('.hip'):
            continue
        text = open(os.path.join(csrc, f)).read()
        n = len(re.findall(r'>>>\s*\(', text))
        c = len(re.findall(r'SV_LAUNCHED\("', text))
        assert n == c, f'{f}: {n} launches, {c} SV_LAUNCHED checks'
        launches += n
        checked += c
    assert launches >= 70
    assert 'sv::launch_failed' in _dynamic_symbols(False)
