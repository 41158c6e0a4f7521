"""Host-side API of the MI355X chunker: one ``GpuChunker`` per (key, min, max, device).

Mirrors the reference's chunker object (``_replicat_adapters._gclmulchunker``,
/root/reference/src/adapters.cpp:16-40) and adds the batch entry points of the C ABI:

* ``next_cut(buffer, final)``          -- exactly adapters.cpp:42-70 on a host buffer;
* ``chunk_device(...)``                -- many device-resident streams, results left in HBM;
* ``chunk_host(buffers, last_piece)``  -- many host streams, pinned copies in, cuts back out.

Streams follow replicat's piece framing (adapters.py:290-305): a stream of L bytes whose last
piece starts at byte P is cut exactly as replicat's adapter loop cuts those pieces.
"""
import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import (RC_OPEN, RC_PIPELINE_END, RC_PIPELINED, ChunkerError, ChunkerFault, check,
                   check_counts, lib)

MIN_LENGTH = 128_000     # replicat/utils/adapters.py:259
MAX_LENGTH = 5_120_000   # replicat/utils/adapters.py:260


def normalize_params(params):
    """Chunker key from repository params: replicat/utils/adapters.py:280-285."""
    if not params:
        return b'\xff' * 16
    params = bytes(params)
    while len(params) < 16:
        params += params
    return params[:16]


def _ptr_array(values):
    return np.ascontiguousarray(np.asarray(values, dtype=np.uint64))


class GpuChunker:
    """A chunker bound to one HIP device (default: the current one)."""

    def __init__(self, min_length, max_length, key, device=None):
        key = bytes(key)
        if device is None:
            device = _current_device()
        handle = ctypes.c_void_p()
        check(lib().rc_chunker_create(min_length, max_length, key, len(key), int(device),
                                      ctypes.byref(handle)))
        self._h = handle
        self.min_length = int(min_length)
        self.max_length = int(max_length)
        self.device = int(device)

    def close(self):
        h, self._h = getattr(self, '_h', None), None
        if h:
            lib().rc_chunker_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------------- single buffer

    def next_cut(self, data: np.ndarray, final: bool) -> int:
        """adapters.cpp:42-70 on the bytes of a uint8 array (host memory)."""
        out = ctypes.c_uint64()
        check(lib().rc_next_cut(self._h, data.ctypes.data if data.size else None, data.size,
                                1 if final else 0, ctypes.byref(out)))
        return out.value

    # ------------------------------------------------------------------------- batches

    def capacity(self, lens):
        lens = _ptr_array(lens)
        caps = np.zeros(len(lens), dtype=np.uint64)
        total = lib().rc_cut_capacity(self._h, len(lens), lens.ctypes.data, caps.ctypes.data)
        return int(total), caps

    def chunk_device(self, ptrs, lens, last_piece, cuts_ptr, counts_ptr, stream=0, open_=False,
                     pipelined=False, end=False):
        """Enqueue the chunking of device-resident streams (raw device pointers) on a HIP
        stream; cut END offsets land in the device array at ``cuts_ptr`` (u64, per-stream
        regions of ``capacity(lens)`` entries) and counts at ``counts_ptr`` (int64).

        ``pipelined=True`` (RC_PIPELINED): the kernels run on the chunker's CU-partitioned
        streams, this call's chain beside the next call's tile kernel; ``stream`` orders the
        inputs only, and ``wait(stream)`` orders the outputs.  Keep the input and output
        tensors alive until then: torch's caching allocator sees only ``stream``.  ``end``
        (RC_PIPELINE_END): the end of a pipelined sequence -- the chain runs on every CU.

        The counts are the call's error report: read them back through ``check_counts`` (or
        ``counts_host``) before using a cut -- a negative count is a capacity overflow or, for
        every stream of the call, RC_COUNT_FAULT (the tile kernel's fail-safe stop)."""
        ptrs, lens = _ptr_array(ptrs), _ptr_array(lens)
        last = _ptr_array(last_piece if last_piece is not None else np.zeros(len(lens)))
        flags = ((RC_OPEN if open_ else 0) | (RC_PIPELINED if pipelined else 0)
                 | (RC_PIPELINE_END if pipelined and end else 0))
        check(lib().rc_chunk_device(self._h, len(lens), ptrs.ctypes.data, lens.ctypes.data,
                                    last.ctypes.data, flags, cuts_ptr, counts_ptr, stream or None))

    def overlap(self, reserve_cus=0):
        """CUs kept for the chain kernels of pipelined calls (0 = the default); returns the
        split in force."""
        check(lib().rc_chunker_overlap(self._h, int(reserve_cus)))
        return int(lib().rc_chunker_overlap_cus(self._h))

    def overlap_cus(self):
        """CUs reserved for pipelined chains (0 until the first pipelined call sets them up,
        or when the CU-masked streams could not be created)."""
        return int(lib().rc_chunker_overlap_cus(self._h))

    def pipelined_calls(self):
        """Pipelined requests so far that ran on the two streams (the others in sequence)."""
        return int(lib().rc_chunker_pipelined_calls(self._h))

    def check(self):
        """Wait for every call so far and raise ChunkerFault if any call since the last check
        took the tile kernel's fail-safe stop (a workgroup grab never published:
        rc_chunker_check)."""
        check(lib().rc_chunker_check(self._h))

    def wait(self, stream=0):
        """Make a HIP stream wait for every call so far (pipelined or not)."""
        check(lib().rc_chunk_wait(self._h, stream or None))

    def chunk_host(self, buffers, last_piece=None, open_=False):
        """Chunk host streams (uint8 arrays / bytes-like); returns a list of cut-END arrays."""
        arrs = [np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b
                for b in buffers]
        n = len(arrs)
        if n == 0:
            return []
        lens = _ptr_array([a.size for a in arrs])
        ptrs = _ptr_array([a.ctypes.data if a.size else 0 for a in arrs])
        last = _ptr_array(last_piece if last_piece is not None else np.zeros(n))
        total, caps = self.capacity(lens)
        cuts = np.zeros(max(total, 1), dtype=np.uint64)
        counts = np.zeros(n, dtype=np.int64)
        check(lib().rc_chunk_host(self._h, n, ptrs.ctypes.data, lens.ctypes.data,
                                  last.ctypes.data, RC_OPEN if open_ else 0, cuts.ctypes.data,
                                  counts.ctypes.data))
        base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
        return [cuts[b:b + c] for b, c in zip(base, counts)]

    def tile_records(self, ptrs, lens, last_piece=None, groups=False):
        """(keys, js) of the per-tile phase over device streams (inspection / tests); with
        groups=True also the per-quarter group bounds (keys, js, gmax, ghot, hot threshold):
        see rc_tile_records in include/replicat_chunker.h."""
        ptrs, lens = _ptr_array(ptrs), _ptr_array(lens)
        last = _ptr_array(last_piece if last_piece is not None else np.zeros(len(lens)))
        nt = ctypes.c_uint64()
        check(lib().rc_tile_records(self._h, len(lens), ptrs.ctypes.data, lens.ctypes.data,
                                    last.ctypes.data, None, None, None, None, 0,
                                    ctypes.byref(nt)))
        keys = np.zeros(max(nt.value, 1), dtype=np.uint64)
        js = np.zeros(max(nt.value, 1), dtype=np.uint64)
        gm = np.zeros(max(nt.value, 1), dtype=np.uint64)
        gh = np.zeros((max(nt.value, 1), 4), dtype=np.uint64)
        check(lib().rc_tile_records(self._h, len(lens), ptrs.ctypes.data, lens.ctypes.data,
                                    last.ctypes.data, keys.ctypes.data, js.ctypes.data,
                                    gm.ctypes.data, gh.ctypes.data, nt.value, ctypes.byref(nt)))
        if groups:
            return (keys[:nt.value], js[:nt.value], gm[:nt.value], gh[:nt.value],
                    int(lib().rc_group_hot_threshold(self._h)))
        return keys[:nt.value], js[:nt.value]

    # ---------------------------------------------------------------------- profiling

    def read_probe(self, ptr, nbytes, out_ptr, stream=0):
        """rc_read_probe under this chunker's tile schedule (its RC_TILE_* knobs)."""
        check(lib().rc_chunker_read_probe(self._h, ptr, nbytes, out_ptr, stream or None))

    def timing(self, enable: bool):
        check(lib().rc_timing_enable(self._h, 1 if enable else 0))

    def read_timing(self):
        """(tile + edge ms, chain ms, calls) summed since the last read."""
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        check(lib().rc_timing_read(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        return a.value, b.value, n.value

    def read_kernel_timing(self):
        """(tile ms, edge ms, chain ms, calls) summed since the last read (HIP events on the
        launch stream)."""
        t, e, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_uint64()
        check(lib().rc_timing_read_kernels(self._h, ctypes.byref(t), ctypes.byref(e),
                                           ctypes.byref(c), ctypes.byref(n)))
        return t.value, e.value, c.value, n.value


class QueueStream:
    """A HIP stream with a hardware queue of its own (rc_stream_create): kernels on it never
    wait behind another stream's kernels on a shared queue, whatever GPU_MAX_HW_QUEUES is.  A
    BLOCKING stream (CU-masked), so keep the legacy NULL stream out of the work it overlaps.
    ``torch`` gives a torch.cuda.ExternalStream over it.

    Lifetime: torch's caching allocator records events on the streams a tensor was used on
    (``record_stream``) when it frees the tensor, possibly much later, so a stream torch has
    seen must outlive every such tensor (round 4: a destroyed stream crashed a later test).
    Take streams from the process-wide pool (``QueueStream.acquire`` / ``release``): pooled
    streams are reused, never destroyed while the process runs, and released by the library's
    exit hook after Python's own finalisation.  ``close()`` destroys a stream at once only if
    torch never wrapped it (``torch`` never taken); a wrapped stream goes back to the pool under
    a fresh wrapper instead (safe to reuse, not to destroy: the next ``acquire`` hands it out, and
    the exit hook destroys it like the other pooled ones), so closing wrapped streams in a loop
    keeps at most as many streams -- and hardware queues -- as were ever in use at once
    (INTEGRATION §7)."""

    _pool = {}
    _lock = threading.Lock()

    def __init__(self, device=None):
        if device is None:
            device = _current_device()
        h = ctypes.c_void_p()
        check(lib().rc_stream_create(int(device), ctypes.byref(h)))
        self.handle, self.device = h.value, int(device)
        self._torch = None
        self._wrapped = False  # torch has seen this stream (it may record events on it)
        self._pooled = False

    @classmethod
    def acquire(cls, device=None):
        """A pooled stream of `device` (a new one when none is free)."""
        if device is None:
            device = _current_device()
        with cls._lock:
            free = cls._pool.setdefault(int(device), [])
            if free:
                qs = free.pop()
                qs._pooled = False
                return qs
        return cls(device)

    def release(self):
        """Back to the pool (the caller's work on it may still be queued: the next user's work
        follows it in stream order).  Releasing twice pools it once."""
        with QueueStream._lock:
            if self.handle and not self._pooled:
                self._pooled = True
                QueueStream._pool.setdefault(self.device, []).append(self)

    @property
    def torch(self):
        if self.handle is None:
            raise RuntimeError('QueueStream is closed')
        if self._torch is None:
            import torch
            self._torch = torch.cuda.ExternalStream(self.handle, device=self.device)
            self._wrapped = True
        return self._torch

    def close(self):
        """Done with this object for good.  The stream is destroyed now if torch never wrapped
        it; otherwise (torch may still record an event on it when it frees a tensor used there)
        it returns to the pool under a fresh wrapper, and this object is closed."""
        with QueueStream._lock:
            if self._pooled:
                QueueStream._pool[self.device].remove(self)
                self._pooled = False
            h, self.handle = self.handle, None
            if h and self._wrapped:
                qs = QueueStream.__new__(QueueStream)
                qs.handle, qs.device = h, self.device
                qs._torch, qs._wrapped, qs._pooled = self._torch, True, True
                QueueStream._pool.setdefault(self.device, []).append(qs)
                h = None
        self._torch = None
        if h:
            lib().rc_stream_destroy(h)


def tile_keys():
    return lib().rc_tile_keys()


def build_id():
    """The loaded library's build id (replicat_amd/build.py: hash of sources and flags)."""
    return lib().rc_build_id().decode()


def keys_needed(max_length, L, P):
    return lib().rc_keys_needed(max_length, L, P)


def fill_splitmix(ptr, nbytes, seed, stream_id, hip_stream=0):
    check(lib().rc_fill_splitmix(ptr, nbytes, seed, stream_id, hip_stream or None))


def fill_splitmix_streams(ptr, n, nbytes, slot, seed, first_id, id_step=1, hip_stream=0):
    """n synthetic streams of nbytes at ptr + k * slot (ids first_id + k * id_step), one launch."""
    check(lib().rc_fill_splitmix_streams(ptr, n, nbytes, slot, seed, first_id, id_step,
                                         hip_stream or None))


def fill_splitmix_at(ptr, nbytes, seed, stream_id, word0, hip_stream=0):
    check(lib().rc_fill_splitmix_at(ptr, nbytes, seed, stream_id, word0, hip_stream or None))


def read_probe(ptr, nbytes, out_ptr, hip_stream=0):
    check(lib().rc_read_probe(ptr, nbytes, out_ptr, hip_stream or None))


def tables_key(key16, ds):
    ds = _ptr_array(ds)
    out = np.zeros(len(ds), dtype=np.uint64)
    top = np.zeros(len(ds), dtype=np.uint32)
    check(lib().rc_tables_key(bytes(key16), len(ds), ds.ctypes.data, out.ctypes.data,
                              top.ctypes.data))
    return out, top


def _current_device():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.current_device()
    except Exception:  # torch is optional plumbing
        pass
    return 0


def counts_host(counts_tensor):
    """A device counts tensor (int64, torch) read back to a numpy array, checked
    (check_counts): the safe way to consume rc_chunk_device's counts."""
    c = counts_tensor.cpu().numpy()
    check_counts(c)
    return c


__all__ = ['GpuChunker', 'QueueStream', 'normalize_params', 'keys_needed', 'fill_splitmix', 'tables_key',
           'check_counts', 'counts_host', 'ChunkerError', 'ChunkerFault', 'MIN_LENGTH', 'MAX_LENGTH',
           '_lib']
