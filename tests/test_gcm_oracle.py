"""The AES-GCM oracle (oracle/aesgcm_oracle.c) pinned on the CPU.

Known answers: FIPS 197 Appendix C (AES-128/192/256 of one block) and the SP 800-38D test
vectors of McGrew & Viega (test cases 1, 2, 13, 14).  Fixtures: tests/golden/gcm.json, made by
tests/golden/make_gcm_golden.py with the host's OpenSSL libcrypto -- the library `cryptography`'s
AESGCM binds, which replicat's aes_gcm adapter calls (replicat/utils/adapters.py:127-144)."""
import hashlib
import random

import pytest

import golden_util as G

FIPS197 = [  # key, plaintext, ciphertext
    ('000102030405060708090a0b0c0d0e0f', '00112233445566778899aabbccddeeff',
     '69c4e0d86a7b0430d8cdb78070b4c55a'),
    ('000102030405060708090a0b0c0d0e0f1011121314151617', '00112233445566778899aabbccddeeff',
     'dda97ca4864cdfe06eaf70a0ec0d7191'),
    ('000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f',
     '00112233445566778899aabbccddeeff', '8ea2b7ca516745bfeafc49904b496089'),
]

GCM_KAT = [  # key, iv, plaintext, C || T (McGrew & Viega test cases 1, 2, 13, 14)
    ('00' * 16, '00' * 12, '', '58e2fccefa7e3061367f1d57a4e7455a'),
    ('00' * 16, '00' * 12, '00' * 16,
     '0388dace60b6a392f328c2b971b2fe78' 'ab6e47d42cec13bdf53a67b21257bddf'),
    ('00' * 32, '00' * 12, '', '530f8afbc74536b9a963b4f1c4cb738b'),
    ('00' * 32, '00' * 12, '00' * 16,
     'cea7403d4d606b6e074ec5d3baf39d18' 'd0d1c8a799996bf0265b98b5d48ab919'),
]

GCM = G.load('gcm.json')


def plaintext(case):
    if 'pt' in case:
        return bytes.fromhex(case['pt'])
    return random.Random(case['pt_seed']).randbytes(case['pt_len'])


@pytest.mark.parametrize('key,pt,ct', FIPS197)
def test_fips197(oracle, key, pt, ct):
    assert oracle.aes_block(bytes.fromhex(key), bytes.fromhex(pt)).hex() == ct


@pytest.mark.parametrize('key,iv,pt,out', GCM_KAT)
def test_sp800_38d_vectors(oracle, key, iv, pt, out):
    k, v, p = bytes.fromhex(key), bytes.fromhex(iv), bytes.fromhex(pt)
    assert oracle.gcm_encrypt(k, v, p).hex() == out
    assert oracle.gcm_decrypt(k, v, bytes.fromhex(out)) == p


@pytest.mark.parametrize('case', [c for c in GCM['cases'] if c.get('pt_len', 0) <= 200_000],
                         ids=lambda c: c['name'])
def test_openssl_fixtures(oracle, case):
    key, iv, pt = bytes.fromhex(case['key']), bytes.fromhex(case['iv']), plaintext(case)
    out = oracle.gcm_encrypt(key, iv, pt)
    if 'out' in case:
        assert out.hex() == case['out']
    else:
        assert hashlib.sha256(out).hexdigest() == case['out_sha256']
        assert out[-16:].hex() == case['tag']
    assert oracle.gcm_decrypt(key, iv, out) == pt


def test_fixture_set_covers_the_edges():
    names = {c['name'] for c in GCM['cases']}
    for kb in (16, 24, 32):
        for ivn in (8, 12, 13, 16, 60, 128):
            assert f'k{kb}_iv{ivn}_p0' in names and f'k{kb}_iv{ivn}_p16385' in names
    assert any(c.get('pt_len') == 5_120_000 for c in GCM['cases'])


def test_decrypt_rejects_tampering(oracle):
    rnd = random.Random(9)
    key, iv, pt = rnd.randbytes(32), rnd.randbytes(12), rnd.randbytes(1000)
    blob = oracle.gcm_encrypt(key, iv, pt)
    for pos in (0, 500, 999, 1000, 1015):
        bad = bytearray(blob)
        bad[pos] ^= 1
        with pytest.raises(ValueError):
            oracle.gcm_decrypt(key, iv, bytes(bad))
    with pytest.raises(ValueError):
        oracle.gcm_decrypt(rnd.randbytes(32), iv, blob)


def test_gf_mul_algebra(oracle):
    """Field laws of the SP 800-38D product: the identity is 0x80 || 0^120, the product
    commutes and distributes over XOR."""
    rnd = random.Random(4)
    one = b'\x80' + bytes(15)
    for _ in range(20):
        x, y, z = rnd.randbytes(16), rnd.randbytes(16), rnd.randbytes(16)
        assert oracle.gf_mul(x, one) == x
        assert oracle.gf_mul(x, y) == oracle.gf_mul(y, x)
        yz = bytes(a ^ b for a, b in zip(y, z))
        rhs = bytes(a ^ b for a, b in zip(oracle.gf_mul(x, y), oracle.gf_mul(x, z)))
        assert oracle.gf_mul(x, yz) == rhs
