"""The drop-in module's surface against the reference binding's recorded behaviour.

tests/golden/surface.json was produced by calling the reference's own `_replicat_adapters`
(built from /root/reference/src/adapters.cpp) with each case.  Cases the reference rejects
before any chunking happens are checked on the CPU (our validation runs before the device is
touched); the rest need the MI355X.
"""
import pytest

import golden_util as G

from replicat_amd import _replicat_adapters as drop_in  # noqa: E402

SURFACE = G.load('surface.json')


def _surface_call(case):
    # the same call recipe the fixture generator used, applied to the drop-in module
    import numpy as np  # noqa: F401
    from golden_surface import surface_call
    return surface_call(drop_in, case['args'], case['call'])


def _check(case):
    if case['error'] is None:
        r = _surface_call(case)
        assert (list(r) if isinstance(r, tuple) else r) == case['result']
    else:
        exc = {'TypeError': TypeError, 'ValueError': ValueError,
               'AttributeError': AttributeError}[case['error']]
        with pytest.raises(exc) as ei:
            _surface_call(case)
        if case.get('message'):
            assert str(ei.value) == case['message']


PRE_DEVICE = [c for c in SURFACE if c['error'] in ('TypeError', 'ValueError') and c['call'] is None
              or c['args'] == 'kw']


@pytest.mark.parametrize('name', [c['name'] for c in PRE_DEVICE])
def test_rejected_before_device(name):
    _check(next(c for c in SURFACE if c['name'] == name))


@pytest.mark.gpu
@pytest.mark.parametrize('name', [c['name'] for c in SURFACE])
def test_surface_on_device(name):
    torch = pytest.importorskip('torch')
    if not torch.cuda.is_available():
        pytest.skip('needs an MI355X')
    _check(next(c for c in SURFACE if c['name'] == name))


def test_module_shape():
    C = drop_in._gclmulchunker
    assert C.__name__ == '_gclmulchunker' and C.__module__ == '_replicat_adapters'
    import _replicat_adapters as top  # the top-level re-export replicat imports
    assert top._gclmulchunker is C
