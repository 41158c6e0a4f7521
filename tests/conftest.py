import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI library)')
    config.addinivalue_line('markers', 'slow: large inputs (minutes on CPU)')


def pytest_collection_modifyitems(config, items):
    # the full-size oracle digests take minutes on the CPU: opt in with RC_SLOW=1
    if os.environ.get('RC_SLOW') == '1':
        return
    skip = pytest.mark.skip(reason='slow: set RC_SLOW=1')
    for item in items:
        if 'slow' in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope='session')
def oracle():
    from oracle import oracle as o
    o.lib()
    return o
