"""Host-side BLAKE2b state records (rc_blake2b_state_init): RFC 7693 §2.8 parameter block and
hashlib.blake2b's argument errors.  No GPU: the call is host-only."""
import hashlib
import struct

import pytest

from replicat_amd.hashing import STATE_BYTES, state_init

IV = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
      0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]


def test_unkeyed_default():
    s = state_init(64)
    assert len(s) == STATE_BYTES
    h = struct.unpack_from('<8Q', s, 0)
    assert h[0] == IV[0] ^ 0x01010040 and list(h[1:]) == IV[1:]
    t, buflen = struct.unpack_from('<QQ', s, 64)
    assert (t, buflen) == (0, 0)
    assert struct.unpack_from('<I', s, 208)[0] == 64


def test_key_salt_person_layout():
    key, salt, person = b'K' * 7, b'S' * 5, b'P' * 16
    s = state_init(32, key=key, salt=salt, person=person)
    h = struct.unpack_from('<8Q', s, 0)
    assert h[0] == IV[0] ^ (0x01010000 | (7 << 8) | 32)
    salt16, person16 = salt + bytes(11), person
    assert h[4] == IV[4] ^ struct.unpack('<Q', salt16[:8])[0]
    assert h[5] == IV[5] ^ struct.unpack('<Q', salt16[8:])[0]
    assert h[6] == IV[6] ^ struct.unpack('<Q', person16[:8])[0]
    assert struct.unpack_from('<QQ', s, 64) == (0, 128)
    assert s[80:80 + 128] == key + bytes(121)


@pytest.mark.parametrize('kw', [dict(key=b'x' * 65), dict(salt=b'x' * 17), dict(person=b'x' * 17),
                                dict(digest_size=0), dict(digest_size=65)])
def test_errors_match_hashlib(kw):
    with pytest.raises(ValueError) as ref:
        hashlib.blake2b(**kw)
    size = kw.pop('digest_size', 64)
    with pytest.raises(ValueError) as got:
        state_init(size, **kw)
    assert str(got.value) == str(ref.value)
