import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and the built libia.so')
    config.addinivalue_line('markers', 'slow: longer CPU-side oracle runs')


@pytest.fixture(scope='session')
def ctx():
    import ia_amd  # noqa: F401
    from ia_amd import _native
    c = _native.Context(0)
    yield c
    c.close()
