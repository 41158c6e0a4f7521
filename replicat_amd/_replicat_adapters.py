"""Drop-in replacement of replicat's native module ``_replicat_adapters``.

Same surface as /root/reference/src/adapters.cpp:80-86 (pybind11 class ``_gclmulchunker``;
type stub stubs/_replicat_adapters.pyi:3-8), same argument rules and the same errors, so
replicat/utils/adapters.py:10,287-299 runs unchanged on top of it:

* ``_gclmulchunker(min_length, max_length, key, /)`` -- positional only; lengths are
  non-negative integers < 2**64 (``__index__``; bool and numpy ints accepted, floats and
  negatives raise TypeError); ``key`` is any buffer whose ITEM count must be 16
  (ValueError "key must contain exactly 16 characters"), then min <= max (ValueError
  "Minimum length is greater than the maximum one"), then k0 != 0 (ValueError "Bad key
  contents") -- adapters.cpp:18-34.
* readonly ``min_length`` / ``max_length`` (AttributeError on assignment) -- :83-84.
* ``next_cut(buffer, final, /) -> int`` -- ``final`` required and positional (bool-like:
  bool, None, numbers); the buffer's item count is its size, its first ``size`` raw bytes
  are chunked -- :42-70.

The scan runs on the MI355X through libreplicat_chunker.so (no CPU fallback).  Unlike the
pybind11 original the GIL is released while the device works.
"""
import operator

import numpy as np

from .chunker import GpuChunker

__all__ = ['_gclmulchunker']

_U64_LIMIT = 1 << 64


def _size_t(value):
    """pybind11's size_t caster: __index__ objects in [0, 2**64), no floats."""
    if isinstance(value, float):
        raise TypeError('incompatible constructor arguments: expected an integer, got float')
    try:
        v = operator.index(value)
    except TypeError:
        raise TypeError(f'incompatible constructor arguments: expected an integer, '
                        f'got {type(value).__name__}') from None
    if v < 0 or v >= _U64_LIMIT:
        raise TypeError(f'incompatible constructor arguments: {v} does not fit size_t')
    return v


def _bool_like(value):
    """pybind11's bool caster in convert mode: bool, None, or a type with __bool__."""
    if value is None:
        return False
    if isinstance(value, (bool, np.bool_)):
        return bool(value)
    if getattr(type(value), '__bool__', None) is None:
        raise TypeError(f'incompatible function arguments: expected bool, got {type(value).__name__}')
    return bool(value)


def _buffer_items(obj, what):
    """(raw bytes as uint8 array, item count) of a buffer-protocol object."""
    try:
        mv = memoryview(obj)
    except TypeError:
        raise TypeError(f'incompatible function arguments: {what} must support the buffer '
                        f'protocol, got {type(obj).__name__}') from None
    items = mv.nbytes // mv.itemsize if mv.itemsize else 0
    if not mv.c_contiguous:
        mv = memoryview(mv.tobytes())  # the original reads such buffers as contiguous (S7 UB)
    raw = np.frombuffer(mv.cast('B') if mv.ndim != 1 or mv.format != 'B' else mv, dtype=np.uint8)
    return raw, items


class _gclmulchunker:
    __slots__ = ('_min_length', '_max_length', '_gpu')

    def __init__(self, min_length, max_length, key, /):
        mn, mx = _size_t(min_length), _size_t(max_length)
        raw, items = _buffer_items(key, 'key')
        if items != 16:  # adapters.cpp:21 checks the item count, not bytes
            raise ValueError('key must contain exactly 16 characters')
        if mn > mx:
            raise ValueError('Minimum length is greater than the maximum one')
        key16 = raw[:16].tobytes() if raw.size >= 16 else raw.tobytes()
        if len(key16) < 16 or int.from_bytes(key16[:8], 'little') == 0:
            raise ValueError('Bad key contents')
        self._min_length, self._max_length = mn, mx
        self._gpu = GpuChunker(mn, mx, key16)

    @property
    def min_length(self):
        return self._min_length

    @property
    def max_length(self):
        return self._max_length

    def next_cut(self, buffer, final, /):
        raw, items = _buffer_items(buffer, 'buffer')
        return self._gpu.next_cut(raw[:items], _bool_like(final))

    def __repr__(self):
        return f'<_replicat_adapters._gclmulchunker object at {id(self):#x}>'


_gclmulchunker.__module__ = '_replicat_adapters'
