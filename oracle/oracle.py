"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The plain-C restatement of replicat's chunker (oracle/gclmul_oracle.c, citing
/root/reference/src/adapters.cpp:18-77 and replicat/utils/adapters.py:274-305).  Imported only
by tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg, always as the
checker or the reported CPU baseline -- never by ``replicat_amd`` (the product path).
Pinned against the reference by tests/test_oracle.py (tests/golden/*.json).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liboracle.so')

_u64 = ctypes.c_uint64
_p = ctypes.c_void_p
_lib = None

ERRORS = {
    1: 'key must contain exactly 16 characters',
    2: 'Minimum length is greater than the maximum one',
    3: 'Bad key contents',
}


def build():
    subprocess.run(['make', '-s', '-C', HERE, 'liboracle.so'], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oc_key.restype = _u64
        L.oc_key.argtypes = [_u64, _u64, _u64]
        L.oc_key_soft.restype = _u64
        L.oc_key_soft.argtypes = [_u64, _u64, _u64]
        L.oc_parse_params.restype = ctypes.c_int
        L.oc_parse_params.argtypes = [_u64, _u64, ctypes.c_char_p, _u64, _p, _p]
        L.oc_next_cut.restype = _u64
        L.oc_next_cut.argtypes = [_u64, _u64, _u64, _u64, _p, _u64, ctypes.c_int]
        L.oc_chunk_stream.restype = ctypes.c_int64
        L.oc_chunk_stream.argtypes = [_u64, _u64, _u64, _u64, _p, _u64, _u64, _p, _u64]
        L.oc_keys_needed.restype = _u64
        L.oc_keys_needed.argtypes = [_u64, _u64, _u64]
        L.oc_tile_records.restype = None
        L.oc_tile_records.argtypes = [_u64, _u64, _p, _u64, _u64, _u64, _u64, _p, _p]
        L.oc_tile_groups.restype = None
        L.oc_tile_groups.argtypes = [_u64, _u64, _p, _u64, _u64, _u64, _u64, _u64, _p]
        L.oc_tile_groups_hot.restype = None
        L.oc_tile_groups_hot.argtypes = [_u64, _u64, _p, _u64, _u64, _u64, _u64, _u64, _u64, _p]
        L.oc_chunk_streams_mt.restype = ctypes.c_int
        L.oc_chunk_streams_mt.argtypes = [_u64, _u64, _u64, _u64, _u64, _p, _p, _p, _p, _p,
                                          _p, _p, ctypes.c_int]
        L.oc_fill_splitmix.restype = None
        L.oc_fill_splitmix.argtypes = [_p, _u64, _u64, _u64]
        L.oc_blake2b.restype = ctypes.c_int
        L.oc_blake2b.argtypes = [_p, _u64, ctypes.c_uint32, _p]
        L.oc_blake2b_chunks.restype = ctypes.c_int
        L.oc_blake2b_chunks.argtypes = [_p, _p, _u64, ctypes.c_uint32, _p]
        _cp, _u32 = ctypes.c_char_p, ctypes.c_uint32
        L.oc_aes_block.restype = ctypes.c_int
        L.oc_aes_block.argtypes = [_cp, _u32, _cp, _p]
        L.oc_gcm_encrypt.restype = ctypes.c_int
        L.oc_gcm_encrypt.argtypes = [_cp, _u32, _cp, _u64, _cp, _u64, _p]
        L.oc_gcm_decrypt.restype = ctypes.c_int
        L.oc_gcm_decrypt.argtypes = [_cp, _u32, _cp, _u64, _cp, _u64, _p]
        L.oc_gf_mul.restype = None
        L.oc_gf_mul.argtypes = [_cp, _cp, _p]
        _lib = L
    return _lib


def normalize_params(params):
    """adapters.py:280-285 (S5)."""
    if not params:
        return b'\xff' * 16
    params = bytes(params)
    while len(params) < 16:
        params += params
    return params[:16]


def parse_key(min_length, max_length, key16):
    k0, k1 = _u64(), _u64()
    rc = lib().oc_parse_params(min_length, max_length, bytes(key16), len(key16),
                               ctypes.byref(k0), ctypes.byref(k1))
    if rc:
        raise ValueError(ERRORS[rc])
    return k0.value, k1.value


def _buf(data):
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    # the restatement may read up to 8 bytes past a 4-aligned key offset: pad a private copy
    pad = np.zeros(len(arr) + 16, dtype=np.uint8)
    pad[:len(arr)] = arr
    return pad


def chunk_stream(data, min_length, max_length, params=None, last_piece_start=0):
    """Cut END offsets of one stream (S4 closed form over (L, P))."""
    k0, k1 = parse_key(min_length, max_length, normalize_params(params))
    buf = _buf(data)
    L = len(buf) - 16
    cap = L // 4 + 8
    cuts = np.zeros(cap, dtype=np.uint64)
    n = lib().oc_chunk_stream(min_length, max_length, k0, k1, buf.ctypes.data, L,
                              last_piece_start, cuts.ctypes.data, cap)
    assert n >= 0
    return cuts[:n].tolist()


def chunk_pieces(pieces, min_length, max_length, params=None):
    """Chunk lengths the reference adapter yields for this piece list."""
    pieces = [bytes(p) for p in pieces]
    if not pieces:
        return []
    data = b''.join(pieces)
    P = len(data) - len(pieces[-1])
    ends = chunk_stream(data, min_length, max_length, params, P)
    return [e - s for s, e in zip([0] + ends[:-1], ends)]


def next_cut(data, final, min_length, max_length, params=None):
    k0, k1 = parse_key(min_length, max_length, normalize_params(params))
    buf = _buf(data)
    return lib().oc_next_cut(min_length, max_length, k0, k1, buf.ctypes.data, len(buf) - 16,
                             int(bool(final)))


def key(k0, k1, d):
    return lib().oc_key(k0, k1, d)


def key_soft(k0, k1, d):
    return lib().oc_key_soft(k0, k1, d)


def keys_needed(max_length, L, P):
    return lib().oc_keys_needed(max_length, L, P)


def fill_splitmix(nbytes, seed, stream):
    out = np.zeros(nbytes, dtype=np.uint8)
    lib().oc_fill_splitmix(out.ctypes.data, nbytes, seed, stream)
    return out


def chunk_streams_mt(bufs, lens, pstarts, min_length, max_length, params=None, threads=1):
    """Threaded CPU baseline over many host streams (each buffer padded by >= 8 bytes)."""
    k0, k1 = parse_key(min_length, max_length, normalize_params(params))
    n = len(bufs)
    ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
    L = np.asarray(lens, dtype=np.uint64)
    P = np.asarray(pstarts, dtype=np.uint64)
    cap = L // np.uint64(max(4, (min_length + 3) & ~3)) + np.uint64(8)
    base = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64)
    cuts = np.zeros(int(cap.sum()), dtype=np.uint64)
    counts = np.zeros(n, dtype=np.int64)
    lib().oc_chunk_streams_mt(min_length, max_length, k0, k1, n, ptrs.ctypes.data,
                              L.ctypes.data, P.ctypes.data, base.ctypes.data, cap.ctypes.data,
                              cuts.ctypes.data, counts.ctypes.data, threads)
    return [cuts[int(b):int(b) + int(c)].tolist() for b, c in zip(base, counts)]


def blake2b(data, digest_size=64):
    """oracle/blake2b_oracle.c: RFC 7693 BLAKE2b of `data` (what hashlib.blake2b(data,
    digest_size=...).digest() returns; adapters.py:224-225)."""
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros(64, dtype=np.uint8)
    rc = lib().oc_blake2b(arr.ctypes.data if arr.size else None, arr.size, digest_size,
                          out.ctypes.data)
    if rc:
        raise ValueError('digest_size must be between 1 and 64 bytes')
    return out[:digest_size].tobytes()


def blake2b_chunks(stream, ends, digest_size=64):
    """Digest slots (n x 64 bytes) of the chunks [ends[k-1], ends[k]) of one host stream."""
    arr = np.ascontiguousarray(np.frombuffer(stream, dtype=np.uint8)
                               if not isinstance(stream, np.ndarray) else stream)
    e = np.ascontiguousarray(np.asarray(ends, dtype=np.uint64))
    out = np.zeros((len(e), 64), dtype=np.uint8)
    if len(e):
        assert lib().oc_blake2b_chunks(arr.ctypes.data, e.ctypes.data, len(e), digest_size,
                                       out.ctypes.data) == 0
    return out


def aes_block(key, block):
    """oracle/aesgcm_oracle.c: FIPS 197 AES-{128,192,256} of one 16-byte block."""
    out = ctypes.create_string_buffer(16)
    if lib().oc_aes_block(bytes(key), len(key), bytes(block), out):
        raise ValueError('AES key must be 16, 24 or 32 bytes')
    return out.raw


def gcm_encrypt(key, iv, pt):
    """AESGCM(key).encrypt(iv, pt, None) = C || T (SP 800-38D restated; adapters.py:131-134
    prepends the nonce)."""
    pt = bytes(pt)
    out = ctypes.create_string_buffer(len(pt) + 16)
    rc = lib().oc_gcm_encrypt(bytes(key), len(key), bytes(iv), len(iv), pt, len(pt), out)
    if rc:
        raise ValueError(f'oc_gcm_encrypt failed ({rc})')
    return out.raw


def gcm_decrypt(key, iv, ct_tag):
    """AESGCM(key).decrypt(iv, C || T, None); ValueError('InvalidTag') when the tag fails."""
    ct_tag = bytes(ct_tag)
    if len(ct_tag) < 16:
        raise ValueError('InvalidTag')
    n = len(ct_tag) - 16
    out = ctypes.create_string_buffer(max(n, 1))
    rc = lib().oc_gcm_decrypt(bytes(key), len(key), bytes(iv), len(iv), ct_tag, n, out)
    if rc == 3:
        raise ValueError('InvalidTag')
    if rc:
        raise ValueError(f'oc_gcm_decrypt failed ({rc})')
    return out.raw[:n]


def gf_mul(x, y):
    """The SP 800-38D product of two 16-byte field elements."""
    out = ctypes.create_string_buffer(16)
    lib().oc_gf_mul(bytes(x), bytes(y), out)
    return out.raw
