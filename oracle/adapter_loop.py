"""TEST INFRASTRUCTURE ONLY -- replicat's chunker adapter loop, restated, for the CPU baseline.

``adapter_chunks`` is ``gclmulchunker.__call__`` of /root/reference/replicat/utils/adapters.py
(:274-305) with the native chunker object passed in instead of constructed, so bench.py can time
the reference's own ``_replicat_adapters._gclmulchunker`` (oracle/_ref, compiled from
src/adapters.cpp) under the Python loop replicat runs it in -- bytearray append, one
``next_cut`` per chunk, a ``bytes`` copy of every chunk and a front ``del`` -- on the GPU box,
where the reference tree itself does not exist.  ``harness_rate`` restates the timing rule of
``Repository._benchmark_chunker`` (repository.py:1984-2008): piece generation excluded, garbage
collection disabled (``utils.disable_gc``, utils/__init__.py:270-280).
"""
import gc
import time


def adapter_chunks(native, pieces):
    """adapters.py:290-305: yield the chunks of an iterator of pieces."""
    buffer = bytearray()
    it = iter(pieces)
    chunk = next(it, None)
    while chunk is not None:
        buffer += chunk
        next_chunk = next(it, None)
        while True:
            pos = native.next_cut(buffer, bool(next_chunk is None))
            if not pos:
                break
            yield bytes(buffer[:pos])
            del buffer[:pos]
        chunk = next_chunk


def harness_rate(native, pieces):
    """(bytes, seconds, chunk lengths) of the adapter over pre-built pieces, the way
    _benchmark_chunker times it (generation outside the clock, gc off)."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        t0 = time.perf_counter()
        lengths = [len(c) for c in adapter_chunks(native, pieces)]
        elapsed = time.perf_counter() - t0
    finally:
        if enabled:
            gc.enable()
    return sum(lengths), elapsed, lengths
