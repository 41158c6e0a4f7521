"""Batching shim for replicat's chunker adapter (SURVEY.md §8 f, rank 1).

``gclmulchunker`` is a drop-in for ``replicat.utils.adapters.gclmulchunker``
(/root/reference/replicat/utils/adapters.py:257-308): same constructor, same ``__call__``
contract (an iterator of byte pieces in, an iterator of chunk ``bytes`` out) and the same
chunks for the same pieces.  Instead of one ``next_cut`` per chunk (adapters.py:297-303), it
accumulates pieces into a large host batch and hands the whole batch to the device at once:

* while more pieces follow, the batch is chunked as an OPEN stream (RC_OPEN): the device cuts
  while ``L - s >= max_length`` -- exactly the reference's non-final ``next_cut`` calls -- and
  the uncut tail is carried into the next batch;
* the last batch is chunked with the real framing (L, P = start of the last piece), which
  applies the tail rules of adapters.cpp:48-57 exactly as the reference's final calls do.
"""
import os
from abc import ABC, abstractmethod
from typing import ByteString, Iterator, Optional

import numpy as np

from .chunker import MAX_LENGTH, MIN_LENGTH, GpuChunker, normalize_params

# host bytes gathered before a device call; large enough to amortise the call, small enough
# to keep replicat's memory bound (it reads 16 MiB pieces: repository.py:1413,1440)
DEFAULT_BATCH = 256 << 20

try:  # replicat installed: be one of its chunker adapters (isinstance checks, from_config)
    from replicat.utils.adapters import ChunkerAdapter
except ImportError:  # standalone: the same abstract interface, adapters.py:83-103
    class ChunkerAdapter(ABC):
        @property
        @abstractmethod
        def alignment(self) -> Optional[int]:
            """Return the alignment"""

        @abstractmethod
        def generate_chunking_params(self) -> bytes:
            """Generate chunking params"""

        @abstractmethod
        def __call__(self, chunk_iterator: Iterator[ByteString], *,
                     params: Optional[bytes] = None) -> Iterator[bytes]:
            """Re-chunk the incoming stream of bytes using the provided params"""


class gclmulchunker(ChunkerAdapter):
    MIN_LENGTH = MIN_LENGTH
    MAX_LENGTH = MAX_LENGTH
    alignment = 4

    def __init__(self, *, min_length: int = MIN_LENGTH, max_length: int = MAX_LENGTH,
                 batch_bytes: int = DEFAULT_BATCH) -> None:
        if min_length > max_length:
            raise ValueError(f'Minimum length ({min_length}) is greater '
                             f'than the maximum one ({max_length})')
        self.min_length, self.max_length = min_length, max_length
        self.batch_bytes = max(int(batch_bytes), 2 * max_length + 16)
        self._key = self._gpu = None

    def _chunker(self, key16):
        """The device chunker of the call's key.  One is kept (a repository uses one key), so a
        long-lived adapter does not pile up device tables and staging buffers per key; the
        reference builds a fresh native chunker per __call__ (adapters.py:287-289)."""
        if self._key != key16:
            # the previous chunker is dropped, not closed: a generator of an earlier call may
            # still hold it (GpuChunker.__del__ releases it with its last reference)
            self._gpu = GpuChunker(self.min_length, self.max_length, key16)
            self._key = key16
        return self._gpu

    def close(self):
        """Drop this adapter's device chunker (tables, workspaces, pinned staging).  It is
        released with its last reference (GpuChunker.__del__), not here: a generator of an
        earlier __call__ may still be cutting with it, and must be able to finish."""
        self._gpu, self._key = None, None

    def __call__(self, chunk_iterator: Iterator[ByteString], *,
                 params: Optional[bytes] = None) -> Iterator[bytes]:
        chunker = self._chunker(normalize_params(params))
        buffer = bytearray()
        last_start = 0          # start of the most recent piece inside `buffer`
        it = iter(chunk_iterator)
        piece = next(it, None)
        while piece is not None:
            nxt = next(it, None)
            last_start = len(buffer)
            buffer += piece
            final = nxt is None
            if final or len(buffer) >= self.batch_bytes:
                data = np.frombuffer(buffer, dtype=np.uint8)
                if final:
                    ends = chunker.chunk_host([data], [last_start])[0]
                else:
                    ends = chunker.chunk_host([data], open_=True)[0]
                prev = 0
                for e in ends.tolist():
                    yield bytes(buffer[prev:e])
                    prev = e
                del data
                del buffer[:prev]
            piece = nxt

    def generate_chunking_params(self) -> bytes:
        return os.urandom(16)
