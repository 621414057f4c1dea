import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


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
