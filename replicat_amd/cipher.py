"""AES-GCM chunk encryption on the device.

replicat's snapshot loop encrypts every chunk of an encrypted repository with its own subkey
(/root/reference/replicat/repository.py:1470-1473)::

    encrypted_contents = self.props.encrypt(output_chunk, self.props.derive_shared_subkey(digest))

``derive_shared_subkey`` is ``blake2b(length=key_bytes).derive(shared_key, context=digest,
params=shared_kdf_params)`` (repository.py:132-137; replicat/utils/adapters.py:205-213 -- on the
device: ``GpuBlake2b.derive_chunks``), and the default cipher is ``aes_gcm(key_bits=256,
nonce_bits=96)`` (adapters.py:151-158; repository.py:216) whose encrypt / decrypt are
(adapters.py:131-144)::

    nonce = os.urandom(nonce_bytes); return nonce + AESGCM(key).encrypt(nonce, data, None)
    AESGCM(key).decrypt(data[:nonce_bytes], data[nonce_bytes:], None)  # InvalidTag -> DecryptionError

``GpuAesGcm`` mirrors that adapter -- ``key_bytes``, ``generate_key()``, ``encrypt(data, key)``,
``decrypt(data, key)``, ``ValueError('Invalid key size')``, ``DecryptionError`` -- over
include/replicat_cipher.h, and adds batch entry points over host buffers (``encrypt_many`` /
``decrypt_many``), device buffers (``encrypt_device`` / ``decrypt_device``) and the chunks a
``GpuChunker`` left in HBM (``encrypt_chunks``).  Nonces come from ``os.urandom`` on the host, as
in the reference.  There is no CPU fallback: without the HIP library every call raises.
"""
import ctypes
import os

import numpy as np

from ._lib import RC_ERR_TAG, check, last_error, lib
from .chunker import _current_device, _ptr_array

TAG_BYTES = 16


class DecryptionError(Exception):
    """replicat.exceptions.DecryptionError, which the adapter raises for cryptography's
    InvalidTag (adapters.py:141-144)."""


def _bytes(v):
    try:
        return bytes(memoryview(v))
    except TypeError:
        raise TypeError(f"a bytes-like object is required, not '{type(v).__name__}'") from None


def _check_key(key):
    if len(key) not in (16, 24, 32):
        raise ValueError('AESGCM key must be 128, 192, or 256 bits.')


class GpuAesGcm:
    """``aes_gcm(key_bits=..., nonce_bits=...)`` (adapters.py:151-158) on one HIP device."""

    def __init__(self, *, key_bits: int = 256, nonce_bits: int = 96, device=None):
        if key_bits not in (128, 192, 256):
            raise ValueError('Invalid key size')
        self.key_bits, self.nonce_bits = key_bits, nonce_bits
        self._key_bytes, self._nonce_bytes = key_bits // 8, nonce_bits // 8
        self.device = int(_current_device() if device is None else device)
        self._handles = {}

    @property
    def key_bytes(self) -> int:
        return self._key_bytes

    @property
    def nonce_bytes(self) -> int:
        return self._nonce_bytes

    def generate_key(self) -> bytes:
        """CipherAdapter.generate_key (adapters.py:31-32)."""
        return os.urandom(self._key_bytes)

    def handle(self, key_bytes=None):
        """The native handle for keys of ``key_bytes`` (AESGCM accepts any of 16 / 24 / 32 bytes,
        whatever ``key_bits`` says).  Created on first use, so a bad nonce size raises AESGCM's
        ValueError at the first encrypt / decrypt, as in the reference."""
        kb = self._key_bytes if key_bytes is None else int(key_bytes)
        h = self._handles.get(kb)
        if h is None:
            h = ctypes.c_void_p()
            bits = self.nonce_bits if isinstance(self.nonce_bits, int) and 0 <= self.nonce_bits < 1 << 32 else 0
            check(lib().rc_gcm_create(8 * kb, bits, self.device, ctypes.byref(h)))
            self._handles[kb] = h
        return h

    def close(self):
        handles, self._handles = getattr(self, '_handles', {}), {}
        for h in handles.values():
            lib().rc_gcm_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ host buffers

    def encrypt(self, data, key) -> bytes:
        """adapters.py:131-134: nonce || C || T with a fresh os.urandom nonce."""
        return self.encrypt_many([data], [key])[0]

    def decrypt(self, data, key) -> bytes:
        """adapters.py:136-144: DecryptionError when the tag does not verify."""
        return self.decrypt_many([data], [key])[0]

    def encrypt_many(self, datas, keys, nonces=None):
        datas = [_bytes(d) for d in datas]
        keys = [_bytes(k) for k in keys]
        if len(keys) != len(datas):
            raise ValueError('one key per message')
        if nonces is None:
            nonces = [os.urandom(self._nonce_bytes) for _ in datas]
        nonces = [_bytes(v) for v in nonces]
        if len(nonces) != len(datas):
            raise ValueError('one nonce per message')
        for k in keys:
            _check_key(k)
        out = [None] * len(datas)
        for kb in sorted({len(k) for k in keys}):
            idx = [i for i, k in enumerate(keys) if len(k) == kb]
            h = self.handle(kb)
            for i in idx:
                if len(nonces[i]) != self._nonce_bytes:
                    raise ValueError(f'nonce must be {self._nonce_bytes} bytes')
            ins = [np.frombuffer(datas[i], dtype=np.uint8) for i in idx]
            ks = [np.frombuffer(keys[i], dtype=np.uint8) for i in idx]
            ns = [np.frombuffer(nonces[i], dtype=np.uint8) for i in idx]
            outs = [np.empty(self._nonce_bytes + a.size + TAG_BYTES, dtype=np.uint8) for a in ins]
            # the pointer arrays stay referenced for the whole call
            arrs = (_ptr_array([a.ctypes.data if a.size else 0 for a in ins]),
                    _ptr_array([a.size for a in ins]), _ptr_array([a.ctypes.data for a in ks]),
                    _ptr_array([a.ctypes.data for a in ns]), _ptr_array([a.ctypes.data for a in outs]))
            check(lib().rc_gcm_encrypt_host(h, len(idx), *[a.ctypes.data for a in arrs]))
            for i, o in zip(idx, outs):
                out[i] = o.tobytes()
        return out

    def decrypt_many(self, blobs, keys):
        blobs = [_bytes(b) for b in blobs]
        keys = [_bytes(k) for k in keys]
        if len(keys) != len(blobs):
            raise ValueError('one key per message')
        for k in keys:
            _check_key(k)
        over = self._nonce_bytes + TAG_BYTES
        out = [None] * len(blobs)
        for kb in sorted({len(k) for k in keys}):
            idx = [i for i, k in enumerate(keys) if len(k) == kb]
            h = self.handle(kb)
            ins = [np.frombuffer(blobs[i], dtype=np.uint8) for i in idx]
            ks = [np.frombuffer(keys[i], dtype=np.uint8) for i in idx]
            outs = [np.empty(max(a.size - over, 1), dtype=np.uint8) for a in ins]
            ok = np.zeros(len(idx), dtype=np.uint8)
            arrs = (_ptr_array([a.ctypes.data if a.size else 0 for a in ins]),
                    _ptr_array([a.size for a in ins]), _ptr_array([a.ctypes.data for a in ks]),
                    _ptr_array([a.ctypes.data for a in outs]))
            rc = lib().rc_gcm_decrypt_host(h, len(idx), *[a.ctypes.data for a in arrs],
                                           ok.ctypes.data)
            if rc not in (0, RC_ERR_TAG):
                check(rc)
            for j, i in enumerate(idx):
                if not ok[j]:
                    raise DecryptionError(f'message {i}: {last_error() or "InvalidTag"}')
                out[i] = outs[j][:max(ins[j].size - over, 0)].tobytes()
        return out

    # ---------------------------------------------------------------- device buffers

    def encrypt_device(self, in_ptrs, lens, key_ptrs, nonce_ptrs, out_ptrs, stream=0):
        """Enqueue encrypt of device buffers: out_ptrs[i] receives nonce || C || T."""
        ins, lens, ks, ns, outs = (_ptr_array(v) for v in (in_ptrs, lens, key_ptrs, nonce_ptrs,
                                                           out_ptrs))
        check(lib().rc_gcm_encrypt_device(self.handle(), len(lens), ins.ctypes.data,
                                          lens.ctypes.data, ks.ctypes.data, ns.ctypes.data,
                                          outs.ctypes.data, stream or None))

    def decrypt_device(self, in_ptrs, lens, key_ptrs, out_ptrs, ok_ptr, stream=0):
        """Enqueue decrypt of device blobs nonce || C || T (lens: whole blobs); ok_ptr receives
        one byte per blob, 1 when its tag verifies."""
        ins, lens, ks, outs = (_ptr_array(v) for v in (in_ptrs, lens, key_ptrs, out_ptrs))
        check(lib().rc_gcm_decrypt_device(self.handle(), len(lens), ins.ctypes.data,
                                          lens.ctypes.data, ks.ctypes.data, outs.ctypes.data,
                                          ok_ptr, stream or None))

    def chunks_layout(self, chunker, lens):
        """(total bytes, per-stream offsets) of encrypt_chunks' output buffer: chunk k of stream i
        (cut range [s, e)) lands at base[i] + s + k (nonce_bytes + 16)."""
        lens = _ptr_array(lens)
        base = np.zeros(len(lens), dtype=np.uint64)
        total = lib().rc_gcm_chunks_layout(self.handle(), chunker._h, len(lens), lens.ctypes.data,
                                           base.ctypes.data)
        return int(total), base

    def encrypt_chunks(self, chunker, ptrs, lens, cuts_ptr, counts_ptr, keys_ptr, nonces_ptr,
                       out_ptr, stream=0):
        """Enqueue encrypt(chunk, subkey) of every chunk ``chunker.chunk_device`` wrote for these
        streams (repository.py:1470-1473): cut slot c takes the key at keys + 64 c and the nonce at
        nonces + nonce_bytes c; blobs land as ``chunks_layout`` says."""
        ptrs, lens = _ptr_array(ptrs), _ptr_array(lens)
        check(lib().rc_gcm_encrypt_chunks(self.handle(), chunker._h, len(lens), ptrs.ctypes.data,
                                          lens.ctypes.data, cuts_ptr, counts_ptr, keys_ptr,
                                          nonces_ptr, out_ptr, stream or None))

    # ---------------------------------------------------------------------- profiling

    def timing(self, enable: bool):
        check(lib().rc_gcm_timing_enable(self.handle(), 1 if enable else 0))

    def read_timing(self):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        check(lib().rc_gcm_timing_read(self.handle(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


__all__ = ['GpuAesGcm', 'DecryptionError', 'TAG_BYTES']
