"""The BLAKE2b restatement (oracle/blake2b_oracle.c) pinned against RFC 7693's known answer and
against hashlib -- the dependency replicat's `blake2b.digest` calls (replicat/utils/adapters.py
:224-225) -- plus the digest C ABI's host-side checks (no GPU needed)."""
import hashlib
import random

import numpy as np
import pytest

from replicat_amd import _lib

# RFC 7693 Appendix A: BLAKE2b-512("abc")
RFC7693_ABC = bytes.fromhex(
    'ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1'
    '7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923')


def test_rfc7693_known_answer(oracle):
    assert oracle.blake2b(b'abc') == RFC7693_ABC
    assert hashlib.blake2b(b'abc').digest() == RFC7693_ABC


@pytest.mark.parametrize('size', [1, 16, 20, 32, 48, 63, 64])
def test_block_boundaries_vs_hashlib(oracle, size):
    rnd = random.Random(size)
    for n in list(range(0, 300)) + [383, 384, 385, 1023, 1024, 1025]:
        data = rnd.randbytes(n)
        assert oracle.blake2b(data, size) == hashlib.blake2b(data, digest_size=size).digest(), n


def test_random_messages_vs_hashlib(oracle):
    rnd = random.Random(7)
    for _ in range(60):
        n = rnd.choice([rnd.randrange(0, 5000), rnd.randrange(0, 300_000)])
        data = rnd.randbytes(n)
        assert oracle.blake2b(data) == hashlib.blake2b(data).digest()


def test_chunk_slots(oracle):
    rnd = random.Random(3)
    data = rnd.randbytes(100_003)
    ends = [5, 128, 129, 4000, 4001, 77_777, 100_003]
    slots = oracle.blake2b_chunks(data, ends, 32)
    prev = 0
    for k, e in enumerate(ends):
        assert slots[k, :32].tobytes() == hashlib.blake2b(data[prev:e], digest_size=32).digest()
        assert not slots[k, 32:].any()
        prev = e


def test_bad_digest_size(oracle):
    for bad in (0, 65):
        with pytest.raises(ValueError, match='between 1 and 64'):
            oracle.blake2b(b'x', bad)


def test_hasher_rejects_digest_size_like_hashlib():
    """GpuBlake2b(length=...) raises hashlib's ValueError before touching a device."""
    from replicat_amd.hashing import GpuBlake2b
    for bad in (0, 65, -1):
        with pytest.raises(ValueError) as exc:
            GpuBlake2b(length=bad)
        with pytest.raises(ValueError) as ref:
            hashlib.blake2b(digest_size=bad)
        assert str(exc.value).split(' (rc=')[0] == str(ref.value)
    with pytest.raises(TypeError):
        GpuBlake2b(length='a')


def test_hasher_needs_a_device():
    """Without a GPU the product path fails loudly; there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is present')
    from replicat_amd.hashing import GpuBlake2b
    with pytest.raises((_lib.ChunkerUnavailable, _lib.ChunkerError)):
        GpuBlake2b(length=64, device=0)
    assert np.dtype(np.uint8).itemsize == 1
