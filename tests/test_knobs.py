"""The library's environment knobs (replicat_amd/csrc/knobs.h): one table, read once per handle,
range-checked.  CPU only: the chunker reads the table after the reference's own argument checks
(adapters.cpp:21-29) and before it looks for a device, so a malformed knob is reported here as
RC_ERR_ARGUMENT and a legal one gets as far as "no device"."""
import ctypes
import os
import re

import pytest

from replicat_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'replicat_amd', 'csrc')


def _table():
    src = open(os.path.join(CSRC, 'knobs.h')).read()
    return re.findall(r'\{"(RC_[A-Z0-9_]+)", (-?\d+)', src)


def test_getenv_only_in_the_knob_table():
    for name in sorted(os.listdir(CSRC)):
        if name == 'knobs.h' or not name.endswith(('.cpp', '.hip', '.h')):
            continue
        text = open(os.path.join(CSRC, name)).read()
        assert 'getenv' not in text, f'{name} reads the environment outside knobs.h'


def test_every_knob_is_documented():
    doc = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
    names = [n for n, _ in _table()]
    assert len(names) == len(set(names)) >= 15
    for n in names:
        assert n in doc, f'{n} missing from INTEGRATION.md'


def _create():
    h = ctypes.c_void_p()
    rc = _lib.lib().rc_chunker_create(128_000, 5_120_000, b'\xff' * 16, 16, 0, ctypes.byref(h))
    if rc == 0:
        _lib.lib().rc_chunker_destroy(h)
    return rc, _lib.last_error()


@pytest.mark.parametrize('name,value', [
    ('RC_TILE_CHUNK', '1'), ('RC_TILE_CHUNK', '99999'), ('RC_TILE_STATIC', '1001'),
    ('RC_TILE_STATIC', 'ten'), ('RC_LANE_CHAIN', '2'), ('RC_LANE_CHAIN', ''),
    ('RC_SEGMENT_EXT', '-1'), ('RC_PIPE_ALL', 'yes'), ('RC_OVERLAP_CUS', '0'),
    ('RC_TILE_GROUPS', 'on'), ('RC_SEGMENT_BYTES', '12abc')])
def test_malformed_knob_fails_creation(monkeypatch, name, value):
    monkeypatch.setenv(name, value)
    rc, msg = _create()
    assert rc == _lib.RC_ERR_ARGUMENT
    assert name in msg


@pytest.mark.parametrize('name,value', [
    ('RC_TILE_CHUNK', '8'), ('RC_TILE_STATIC', '0x64'), ('RC_LANE_CHAIN', 'lane'),
    ('RC_LANE_CHAIN', 'auto'), ('RC_PIPE_ALL', '1'), ('RC_B2_LANE_MAX', '-1'),
    ('RC_TILE_GROUPS', '0'), ('RC_SEGMENT_BYTES', '65536')])
def test_legal_knob_passes(monkeypatch, name, value):
    monkeypatch.setenv(name, value)
    rc, msg = _create()
    # no GPU in the build container: a legal setting gets as far as the device check
    assert rc in (_lib.RC_OK, _lib.RC_ERR_NO_DEVICE), msg


def test_reference_errors_come_first(monkeypatch):
    """The reference's ValueErrors keep their precedence over a knob error."""
    monkeypatch.setenv('RC_TILE_CHUNK', 'bad')
    h = ctypes.c_void_p()
    assert _lib.lib().rc_chunker_create(10, 5, b'\xff' * 16, 16, 0, ctypes.byref(h)) == \
        _lib.RC_ERR_MIN_GT_MAX
