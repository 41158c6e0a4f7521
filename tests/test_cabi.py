"""The C-ABI library on the CPU: it loads, exports every symbol include/replicat_chunker.h
declares, builds the same key tables as the oracle's clmul, and fails loudly without a GPU."""
import os
import random
import re

import numpy as np
import pytest

from replicat_amd import _lib, chunker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = ''.join(open(os.path.join(ROOT, 'include', h)).read()
                   for h in ('replicat_chunker.h', 'replicat_digest.h', 'replicat_cipher.h'))
    return sorted(set(re.findall(r'^\w[\w\s\*]*?\b(rc_\w+)\s*\(', text, re.M)))


def test_exports_every_declared_symbol():
    syms = header_symbols()
    assert len(syms) >= 15
    assert 'rc_blake2b_chunks' in syms and 'rc_chunk_digest_host' in syms
    lib = _lib.lib()
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f'{s} has no ctypes signature'


def test_abi_version_matches_package():
    import replicat_amd
    v = _lib.lib().rc_version()
    assert '%d.%d.%d' % (v // 10000, v // 100 % 100, v % 100) == replicat_amd.__version__


def test_tables_match_oracle_clmul(oracle):
    rnd = random.Random(11)
    for _ in range(8):
        key = rnd.randbytes(16)
        ds = [rnd.getrandbits(64) for _ in range(500)] + [0, 1, 1 << 63, (1 << 64) - 1]
        out, top = chunker.tables_key(key, ds)
        k0 = int.from_bytes(key[:8], 'little')
        k1 = int.from_bytes(key[8:], 'little')
        exp = [oracle.key_soft(k0, k1, d) for d in ds]
        assert [int(x) for x in out] == exp
        assert [int(t) for t in top] == [e >> 48 for e in exp]


def test_keys_needed_matches_oracle(oracle):
    rnd = random.Random(2)
    for _ in range(2000):
        mx = rnd.choice([1, 4, 5, 8, 100, 5_120_000])
        L = rnd.randrange(0, 40 * mx + 10)
        P = rnd.randrange(0, L + 1)
        assert chunker.keys_needed(mx, L, P) == oracle.keys_needed(mx, L, P)


def test_valid_key_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is present')
    with pytest.raises(_lib.ChunkerUnavailable):
        chunker.GpuChunker(128_000, 5_120_000, b'\xff' * 16)


def test_constructor_errors_in_reference_order():
    with pytest.raises(ValueError, match='exactly 16'):
        chunker.GpuChunker(11, 10, b'\xff' * 3)
    with pytest.raises(ValueError, match='greater than the maximum'):
        chunker.GpuChunker(11, 10, b'\xff' * 16)
    with pytest.raises(ValueError, match='Bad key'):
        chunker.GpuChunker(1, 10, bytes(8) + b'\xff' * 8)


def test_normalize_params():
    assert chunker.normalize_params(None) == b'\xff' * 16
    assert chunker.normalize_params(b'') == b'\xff' * 16
    assert chunker.normalize_params(b'abc') == (b'abc' * 6)[:16]
    assert chunker.normalize_params(b'x' * 40) == b'x' * 16


def test_tile_geometry():
    assert chunker.tile_keys() == 4096
