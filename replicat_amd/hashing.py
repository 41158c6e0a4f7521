"""BLAKE2b chunk digests on the device.

replicat's snapshot loop takes ``self.props.hash_digest(output_chunk)`` of every chunk it cuts
(/root/reference/replicat/repository.py:1462).  The default hashing adapter is
``blake2b(length=64)`` (repository.py:217; replicat/utils/adapters.py:195-197), whose
``digest(data)`` is ``hashlib.blake2b(data, digest_size=length).digest()`` (adapters.py:224-225).

``GpuBlake2b`` mirrors that adapter's unkeyed surface -- ``digest_size`` and ``digest(data)`` --
and adds the batch entry points of include/replicat_digest.h:

* ``digest_many(buffers)``          -- host buffers in, digests out (blocking);
* ``digest_device(ptrs, lens, out)`` -- device buffers, digests left in HBM (64-byte slots);
* ``digest_chunks(chunker, ...)``    -- the chunks a ``GpuChunker.chunk_device`` call left in
  HBM, digested without a host round trip (digest of cut slot s at out + 64 s).

and the incremental / keyed half of the adapter over device-resident states
(``rc_blake2b_state``, include/replicat_digest.h):

* ``state_init(digest_size, key, salt, person)`` -- hashlib.blake2b's parameters, as a 256-byte
  record to copy to the device;
* ``update_device(states, ptrs, lens, finals, out)`` -- many HashlibIncrementalHasher.feed /
  .digest steps (adapters.py:106-114) in one launch: per-file digests (repository.py:1433-1446),
  the shared-subkey KDF ``derive`` (adapters.py:203-211) and ``mac`` (:217-221);
* ``DeviceIncrementalHasher`` -- ``incremental_hasher()`` (adapters.py:227-228) itself;
* ``derive_chunks(...)`` -- the subkey of every chunk digest left in HBM (repository.py:1470-1472).

There is no CPU fallback: without the HIP library every call raises.
"""
import ctypes

import numpy as np

from ._lib import RC_DIGEST_SLOT, check, lib
from .chunker import _current_device, _ptr_array

SLOT = RC_DIGEST_SLOT
STATE_BYTES = 256   # sizeof(rc_blake2b_state)


def _bytes_arg(name, v):
    if v is None:
        return b''
    try:
        return bytes(memoryview(v))
    except TypeError:
        raise TypeError(f"a bytes-like object is required, not '{type(v).__name__}'") from None


def state_init(digest_size: int = 64, *, key=b'', salt=b'', person=b'') -> bytes:
    """hashlib.blake2b(digest_size=..., key=..., salt=..., person=...) before any data, as the
    256-byte rc_blake2b_state record (host memory; copy it to the device to use it).  Raises
    hashlib's ValueErrors for out-of-range sizes."""
    if not isinstance(digest_size, int):
        raise TypeError(f'{type(digest_size).__name__!r} object cannot be interpreted as an integer')
    key, salt, person = (_bytes_arg(n, v) for n, v in (('key', key), ('salt', salt),
                                                        ('person', person)))
    out = ctypes.create_string_buffer(STATE_BYTES)
    check(lib().rc_blake2b_state_init(digest_size if 0 <= digest_size < 1 << 32 else 0,
                                      key or None, len(key), salt or None, len(salt),
                                      person or None, len(person), out))
    return out.raw


class GpuBlake2b:
    """``blake2b(length=...)`` (adapters.py:195-197) on one HIP device."""

    def __init__(self, *, length: int = 64, device=None):
        if device is None:
            device = _current_device()
        if not isinstance(length, int):
            raise TypeError(f'{type(length).__name__!r} object cannot be interpreted as an integer')
        handle = ctypes.c_void_p()
        check(lib().rc_blake2b_create(length if 0 <= length < 1 << 32 else 0, int(device),
                                      ctypes.byref(handle)))
        self._h = handle
        self.digest_size = int(length)
        self.device = int(device)

    def close(self):
        h, self._h = getattr(self, '_h', None), None
        if h:
            lib().rc_blake2b_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ host buffers

    def digest(self, data) -> bytes:
        """adapters.py:224-225 for one host buffer."""
        return self.digest_many([data])[0]

    def digest_many(self, buffers):
        arrs = [np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else
                np.ascontiguousarray(b).view(np.uint8).reshape(-1) for b in buffers]
        n = len(arrs)
        if n == 0:
            return []
        lens = _ptr_array([a.size for a in arrs])
        ptrs = _ptr_array([a.ctypes.data if a.size else 0 for a in arrs])
        out = np.zeros((n, SLOT), dtype=np.uint8)
        check(lib().rc_blake2b_host(self._h, n, ptrs.ctypes.data, lens.ctypes.data,
                                    out.ctypes.data))
        return [out[i, :self.digest_size].tobytes() for i in range(n)]

    # ---------------------------------------------------------------- device buffers

    def digest_device(self, ptrs, lens, out_ptr, stream=0):
        """Enqueue the digests of device buffers (raw pointers) into 64-byte slots at out_ptr."""
        ptrs, lens = _ptr_array(ptrs), _ptr_array(lens)
        check(lib().rc_blake2b_device(self._h, len(lens), ptrs.ctypes.data, lens.ctypes.data,
                                      out_ptr, stream or None))

    def digest_chunks(self, chunker, ptrs, lens, cuts_ptr, counts_ptr, out_ptr, stream=0):
        """Enqueue the digests of the chunks ``chunker.chunk_device`` wrote for these streams:
        the slot of cut s (``cuts_ptr`` layout, ``chunker.capacity(lens)``) is out + 64 s."""
        ptrs, lens = _ptr_array(ptrs), _ptr_array(lens)
        check(lib().rc_blake2b_chunks(self._h, chunker._h, len(lens), ptrs.ctypes.data,
                                      lens.ctypes.data, cuts_ptr, counts_ptr, out_ptr,
                                      stream or None))

    def update_device(self, state_ptrs, ptrs, lens, finals, out_ptr=0, stream=0):
        """Enqueue incremental updates (rc_blake2b_update_device): item i feeds device buffer
        ptrs[i] into the device state state_ptrs[i]; finals[i] also writes its digest to
        out + 64 i (the state is then left as it was)."""
        states, ptrs, lens = _ptr_array(state_ptrs), _ptr_array(ptrs), _ptr_array(lens)
        fin = np.ascontiguousarray(np.asarray(finals, dtype=np.uint8).reshape(-1))
        if not (len(states) == len(ptrs) == len(lens) == len(fin)):
            raise ValueError('states, ptrs, lens and finals differ in length')
        check(lib().rc_blake2b_update_device(self._h, len(lens), states.ctypes.data,
                                             ptrs.ctypes.data, lens.ctypes.data,
                                             fin.ctypes.data, out_ptr or None, stream or None))

    def derive_chunks(self, chunker, lens, counts_ptr, kdf_state_ptr, digests_ptr, keys_ptr,
                      stream=0):
        """Enqueue ``derive_shared_subkey(digest)`` of every chunk digest ``digest_chunks`` left
        in HBM (repository.py:132-137, 1470-1472; adapters.py:205-213): the device state at
        kdf_state_ptr -- ``state_init(key_bytes, key=shared_key, salt=shared_kdf_params)``, only
        read -- absorbs the digest of cut slot s and its digest lands at keys + 64 s."""
        lens = _ptr_array(lens)
        check(lib().rc_blake2b_derive_chunks(self._h, chunker._h, len(lens), lens.ctypes.data,
                                             counts_ptr, kdf_state_ptr, digests_ptr,
                                             self.digest_size, keys_ptr, stream or None))

    # ---------------------------------------------------------------------- profiling

    def timing(self, enable: bool):
        check(lib().rc_blake2b_timing_enable(self._h, 1 if enable else 0))

    def read_timing(self):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        check(lib().rc_blake2b_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


class DeviceIncrementalHasher:
    """``blake2b(length).incremental_hasher()`` (adapters.py:227-228; HashlibIncrementalHasher
    :106-114) with its state in HBM: ``feed(data)`` uploads and compresses on the device,
    ``digest()`` finalises.  Optional key / salt / person as hashlib.blake2b takes them."""

    def __init__(self, hasher: 'GpuBlake2b', *, key=b'', salt=b'', person=b''):
        import torch
        self._hasher = hasher
        dev = torch.device('cuda', hasher.device)
        init = np.frombuffer(state_init(hasher.digest_size, key=key, salt=salt, person=person),
                             dtype=np.uint8)
        self._state = torch.from_numpy(init.copy()).to(dev)
        self._slot = torch.zeros(SLOT, dtype=torch.uint8, device=dev)
        self._dev = dev

    def _run(self, data, final):
        import torch
        arr = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(0, np.uint8)
        buf = torch.from_numpy(arr.copy()).to(self._dev) if arr.size else None
        stream = torch.cuda.current_stream(self._dev).cuda_stream
        self._hasher.update_device([self._state.data_ptr()], [buf.data_ptr() if buf is not None else 0],
                                   [arr.size], [1 if final else 0], self._slot.data_ptr(), stream)
        torch.cuda.current_stream(self._dev).synchronize()

    def feed(self, data) -> None:
        self._run(memoryview(data).cast('B'), False)

    def digest(self) -> bytes:
        self._run(b'', True)
        return self._slot.cpu().numpy()[:self._hasher.digest_size].tobytes()


def chunk_digest_host(chunker, hasher, buffers, last_piece=None, open_=False):
    """The snapshot loop's chunkify + hash_digest over host streams in one device pass
    (rc_chunk_digest_host): returns (cut-END arrays, per-stream (count x digest_size) digests)."""
    from ._lib import RC_OPEN
    arrs = [np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b
            for b in buffers]
    n = len(arrs)
    if n == 0:
        return [], []
    lens = _ptr_array([a.size for a in arrs])
    ptrs = _ptr_array([a.ctypes.data if a.size else 0 for a in arrs])
    last = _ptr_array(last_piece if last_piece is not None else np.zeros(n))
    total, caps = chunker.capacity(lens)
    cuts = np.zeros(max(total, 1), dtype=np.uint64)
    counts = np.zeros(n, dtype=np.int64)
    digests = np.zeros((max(total, 1), SLOT), dtype=np.uint8)
    check(lib().rc_chunk_digest_host(chunker._h, hasher._h, n, ptrs.ctypes.data,
                                     lens.ctypes.data, last.ctypes.data,
                                     RC_OPEN if open_ else 0, cuts.ctypes.data,
                                     counts.ctypes.data, digests.ctypes.data))
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    return ([cuts[b:b + c] for b, c in zip(base, counts)],
            [digests[b:b + c, :hasher.digest_size] for b, c in zip(base, counts)])


__all__ = ['GpuBlake2b', 'DeviceIncrementalHasher', 'chunk_digest_host', 'state_init', 'SLOT',
           'STATE_BYTES']
