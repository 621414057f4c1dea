import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_sessionstart(session):
    """A fresh checkout has no built libsvhip.so (build artefacts stay out of git): build it once, in tree,
    the way __graft_entry__.build() does, so the CPU suite's ABI tests can load it."""
    import shutil
    import subprocess
    lib = os.path.join(ROOT, 'supervillain_amd', 'libsvhip.so')
    if not os.path.exists(lib) and shutil.which('make') and os.path.exists('/opt/rocm/bin/hipcc'):
        subprocess.run(['make', '-j', str(min(8, os.cpu_count() or 1)), '-C', os.path.join(ROOT, 'supervillain_amd', 'csrc')],
                       check=False, capture_output=True)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


@pytest.fixture(scope='session')
def oracle_lib():
    """Build (if needed) and load the CPU oracle.  Test infrastructure only."""
    import subprocess
    lib = os.path.join(ROOT, 'oracle', 'liboracle.so')
    src = os.path.join(ROOT, 'oracle', 'sv_oracle.c')
    if not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src):
        subprocess.run(['make', '-C', os.path.join(ROOT, 'oracle')], check=True, capture_output=True)
    from oracle import oracle
    oracle.lib()
    return oracle
