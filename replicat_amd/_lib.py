"""ctypes binding of the C ABI (include/replicat_chunker.h) -> libreplicat_chunker.so.

There is no fallback: if the in-tree HIP library is missing or cannot be loaded, every entry
point raises ``ChunkerUnavailable``.  Loading the library does not need a GPU; creating a
chunker does (``RC_ERR_NO_DEVICE`` otherwise).
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# RC_LIB_PATH: load a diagnostic build instead (profiling experiments only)
LIB_PATH = os.environ.get('RC_LIB_PATH') or os.path.join(HERE, 'libreplicat_chunker.so')

RC_OK = 0
RC_ERR_KEY_LENGTH = 1
RC_ERR_MIN_GT_MAX = 2
RC_ERR_BAD_KEY = 3
RC_ERR_DIGEST_SIZE = 4
RC_ERR_B2_PARAM = 5
RC_ERR_KEY_SIZE = 6
RC_ERR_NONCE_SIZE = 7
RC_ERR_TAG = 8
RC_ERR_ARGUMENT = 10
RC_ERR_ALIGN = 11
RC_ERR_HIP = 12
RC_ERR_OVERFLOW = 13
RC_ERR_NO_DEVICE = 14
RC_ERR_DEVICE_FAULT = 15
RC_COUNT_OVERFLOW = -1  # rc_chunk_device's per-stream counts besides the cut count
RC_COUNT_FAULT = -3
RC_OPEN = 1
RC_PIPELINED = 2
RC_PIPELINE_END = 4
RC_DIGEST_SLOT = 64

# every symbol include/replicat_chunker.h, replicat_digest.h and replicat_cipher.h declare:
# name -> (restype, argtypes)
_u64, _i64, _u32, _int, _p = ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
SIGNATURES = {
    'rc_version': (_int, []),
    'rc_build_id': (ctypes.c_char_p, []),
    'rc_last_error': (ctypes.c_char_p, []),
    'rc_chunker_create': (_int, [_u64, _u64, _p, _u64, _int, ctypes.POINTER(_p)]),
    'rc_chunker_destroy': (None, [_p]),
    'rc_chunker_min_length': (_u64, [_p]),
    'rc_chunker_max_length': (_u64, [_p]),
    'rc_next_cut': (_int, [_p, _p, _u64, _int, ctypes.POINTER(_u64)]),
    'rc_cut_capacity': (_u64, [_p, _u64, _p, _p]),
    'rc_chunk_device': (_int, [_p, _u64, _p, _p, _p, _u32, _p, _p, _p]),
    'rc_chunk_host': (_int, [_p, _u64, _p, _p, _p, _u32, _p, _p]),
    'rc_chunker_overlap': (_int, [_p, _u32]),
    'rc_chunker_overlap_cus': (_u32, [_p]),
    'rc_chunker_pipelined_calls': (_u64, [_p]),
    'rc_chunker_check': (_int, [_p]),
    'rc_chunk_wait': (_int, [_p, _p]),
    'rc_stream_create': (_int, [_int, ctypes.POINTER(_p)]),
    'rc_stream_destroy': (None, [_p]),
    'rc_timing_enable': (_int, [_p, _int]),
    'rc_timing_read': (_int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(_u64)]),
    'rc_timing_read_kernels': (_int, [_p, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64)]),
    'rc_fill_splitmix': (_int, [_p, _u64, _u64, _u64, _p]),
    'rc_fill_splitmix_at': (_int, [_p, _u64, _u64, _u64, _u64, _p]),
    'rc_fill_splitmix_streams': (_int, [_p, _u64, _u64, _u64, _u64, _u64, _u64, _p]),
    'rc_read_probe': (_int, [_p, _u64, _p, _p]),
    'rc_chunker_read_probe': (_int, [_p, _p, _u64, _p, _p]),
    'rc_keys_needed': (_u64, [_u64, _u64, _u64]),
    'rc_host_key': (_u64, [_p, _u64]),
    'rc_tables_key': (_int, [_p, _u64, _p, _p, _p]),
    'rc_tile_records': (_int, [_p, _u64, _p, _p, _p, _p, _p, _p, _p, _u64, ctypes.POINTER(_u64)]),
    'rc_group_hot_threshold': (_u32, [_p]),
    'rc_tile_keys': (_u64, []),
    'rc_tile_schedule': (_int, [_u64, _u32, _u32, _u32, _u32, _p, _u64, ctypes.POINTER(_u64)]),
    # replicat_digest.h
    'rc_blake2b_create': (_int, [_u32, _int, ctypes.POINTER(_p)]),
    'rc_blake2b_destroy': (None, [_p]),
    'rc_blake2b_digest_size': (_u32, [_p]),
    'rc_blake2b_device': (_int, [_p, _u64, _p, _p, _p, _p]),
    'rc_blake2b_host': (_int, [_p, _u64, _p, _p, _p]),
    'rc_blake2b_chunks': (_int, [_p, _p, _u64, _p, _p, _p, _p, _p, _p]),
    'rc_chunk_digest_host': (_int, [_p, _p, _u64, _p, _p, _p, _u32, _p, _p, _p]),
    'rc_blake2b_state_init': (_int, [_u32, _p, _u32, _p, _u32, _p, _u32, _p]),
    'rc_blake2b_update_device': (_int, [_p, _u64, _p, _p, _p, _p, _p, _p]),
    'rc_blake2b_timing_enable': (_int, [_p, _int]),
    'rc_blake2b_timing_read': (_int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64)]),
    'rc_blake2b_derive_chunks': (_int, [_p, _p, _u64, _p, _p, _p, _p, _u32, _p, _p]),
    # replicat_cipher.h
    'rc_gcm_create': (_int, [_u32, _u32, _int, ctypes.POINTER(_p)]),
    'rc_gcm_destroy': (None, [_p]),
    'rc_gcm_key_bytes': (_u32, [_p]),
    'rc_gcm_nonce_bytes': (_u32, [_p]),
    'rc_gcm_encrypt_device': (_int, [_p, _u64, _p, _p, _p, _p, _p, _p]),
    'rc_gcm_decrypt_device': (_int, [_p, _u64, _p, _p, _p, _p, _p, _p]),
    'rc_gcm_encrypt_host': (_int, [_p, _u64, _p, _p, _p, _p, _p]),
    'rc_gcm_decrypt_host': (_int, [_p, _u64, _p, _p, _p, _p, _p]),
    'rc_gcm_chunks_layout': (_u64, [_p, _p, _u64, _p, _p]),
    'rc_gcm_encrypt_chunks': (_int, [_p, _p, _u64, _p, _p, _p, _p, _p, _p, _p, _p]),
    'rc_gcm_timing_enable': (_int, [_p, _int]),
    'rc_gcm_timing_read': (_int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64)]),
}


class ChunkerUnavailable(RuntimeError):
    """The HIP chunker library is not built or cannot run here."""


class ChunkerError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f'{message} (rc={code})')
        self.code = code


class ChunkerFault(ChunkerError):
    """The tile kernel took its fail-safe stop (RC_ERR_DEVICE_FAULT, RC_COUNT_FAULT): the call's
    cuts are not the reference's and must not be used."""


def check_counts(counts):
    """Raise for the negative per-stream counts of rc_chunk_device (any int sequence or array
    read back from the device): ChunkerFault for RC_COUNT_FAULT, ChunkerError(RC_ERR_OVERFLOW)
    for anything else below 0.  Every reader of device counts calls it before using a cut."""
    import numpy as np
    c = np.asarray(counts).reshape(-1)
    if c.size == 0 or int(c.min()) >= 0:
        return
    if (c == RC_COUNT_FAULT).any():
        raise ChunkerFault(RC_ERR_DEVICE_FAULT, 'tile kernel fail-safe stop: a workgroup grab was '
                           'never published, so the call\'s cuts are not the reference\'s')
    raise ChunkerError(RC_ERR_OVERFLOW, f'stream {int(np.argmax(c < 0))} overflowed its cut capacity')


_lock = threading.Lock()
_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ChunkerUnavailable(
                    f'{LIB_PATH} is missing: build it with `python -m replicat_amd.build` '
                    '(hipcc, gfx950); there is no CPU fallback')
            try:
                L = ctypes.CDLL(LIB_PATH)
            except OSError as e:
                raise ChunkerUnavailable(f'cannot load {LIB_PATH}: {e}') from e
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def last_error():
    msg = lib().rc_last_error()
    return msg.decode('utf-8', 'replace') if msg else ''


def check(code):
    """Raise for a non-zero status: the three constructor errors as the reference's ValueErrors
    (src/adapters.cpp:21-29), everything else as ChunkerError/ChunkerUnavailable."""
    if code == RC_OK:
        return
    msg = last_error()
    if code in (RC_ERR_KEY_LENGTH, RC_ERR_MIN_GT_MAX, RC_ERR_BAD_KEY, RC_ERR_DIGEST_SIZE,
                RC_ERR_B2_PARAM, RC_ERR_KEY_SIZE, RC_ERR_NONCE_SIZE):
        raise ValueError(msg)
    if code == RC_ERR_NO_DEVICE:
        raise ChunkerUnavailable(msg)
    if code == RC_ERR_DEVICE_FAULT:
        raise ChunkerFault(code, msg)
    raise ChunkerError(code, msg)
