"""GPU parity of the AES-GCM chunk encryption (replicat_amd/cipher.py over gcm.hip): replicat's
`aes_gcm` cipher adapter (replicat/utils/adapters.py:117-158) and the encrypted snapshot's
per-chunk subkeys (repository.py:132-137, 1470-1473).

Expected values: tests/golden/gcm.json (OpenSSL libcrypto, what `cryptography`'s AESGCM binds),
the oracle (oracle/aesgcm_oracle.c, pinned by tests/test_gcm_oracle.py) and hashlib.blake2b for
the subkeys.  Runs on an MI355X only (-m gpu)."""
import hashlib
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import golden_util as G  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402
from replicat_amd.cipher import DecryptionError, GpuAesGcm  # noqa: E402
from replicat_amd.hashing import SLOT, GpuBlake2b, state_init  # noqa: E402

GCM = G.load('gcm.json')


def plaintext(case):
    if 'pt' in case:
        return bytes.fromhex(case['pt'])
    return random.Random(case['pt_seed']).randbytes(case['pt_len'])


def dev(data):
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    return torch.from_numpy(arr.copy()).cuda()


@pytest.mark.parametrize('case', GCM['cases'], ids=lambda c: c['name'])
def test_openssl_fixture(case):
    key, iv, pt = bytes.fromhex(case['key']), bytes.fromhex(case['iv']), plaintext(case)
    g = GpuAesGcm(key_bits=8 * len(key), nonce_bits=8 * len(iv))
    blob = g.encrypt_many([pt], [key], [iv])[0]
    assert blob[:len(iv)] == iv
    out = blob[len(iv):]
    if 'out' in case:
        assert out.hex() == case['out']
    else:
        assert hashlib.sha256(out).hexdigest() == case['out_sha256']
        assert out[-16:].hex() == case['tag']
    assert g.decrypt_many([blob], [key])[0] == pt


@pytest.mark.parametrize('kb', [16, 24, 32])
@pytest.mark.parametrize('nb', [12, 8, 16, 13, 60])
def test_batches_vs_oracle(oracle, kb, nb):
    rnd = random.Random(kb * 1000 + nb)
    lens = [rnd.choice([0, 1, 15, 16, 17, 4096, 16383, 16384, 16385, rnd.randrange(0, 5000),
                        rnd.randrange(0, 70000)]) for _ in range(24)]
    datas = [rnd.randbytes(n) for n in lens]
    keys = [rnd.randbytes(kb) for _ in lens]
    nonces = [rnd.randbytes(nb) for _ in lens]
    g = GpuAesGcm(key_bits=8 * kb, nonce_bits=8 * nb)
    blobs = g.encrypt_many(datas, keys, nonces)
    for d, k, v, b in zip(datas, keys, nonces, blobs):
        assert b == v + oracle.gcm_encrypt(k, v, d)
    assert g.decrypt_many(blobs, keys) == datas


def test_reference_adapter_tests(oracle):
    """replicat/tests/test_adapters.py:13-51 with the oracle standing in for AESGCM."""
    for bits in (128, 192, 256):
        key = GpuAesGcm(key_bits=bits, nonce_bits=96).generate_key()
        assert isinstance(key, bytes) and len(key) * 8 == bits
    adapter = GpuAesGcm(key_bits=256, nonce_bits=96)
    key = b'<key>'.ljust(32, b'\x00')
    rv = adapter.encrypt(b'<some data>', key)
    assert rv[12:] == oracle.gcm_encrypt(key, rv[:12], b'<some data>')
    nonce = os.urandom(12)
    ct = oracle.gcm_encrypt(key, nonce, b'<some data>')
    with pytest.raises(DecryptionError):
        adapter.decrypt(nonce + ct, b'<bad key>'.ljust(32, b'\x00'))
    with pytest.raises(DecryptionError):
        adapter.decrypt(b'\x00' + nonce + ct, b'<bad key>'.ljust(32, b'\x00'))
    assert adapter.decrypt(nonce + ct, key) == b'<some data>'


def test_errors_and_tampering():
    with pytest.raises(ValueError, match='Invalid key size'):
        GpuAesGcm(key_bits=100)
    with pytest.raises(ValueError, match='between 8 and 128'):
        GpuAesGcm(key_bits=256, nonce_bits=32).encrypt(b'x', bytes(32))
    g = GpuAesGcm()
    with pytest.raises(ValueError, match='128, 192, or 256'):
        g.encrypt(b'x', bytes(10))
    rnd = random.Random(2)
    key, data = rnd.randbytes(32), rnd.randbytes(50_000)
    blob = g.encrypt(data, key)
    assert g.decrypt(blob, key) == data
    for pos in (0, 11, 12, 30_000, len(blob) - 17, len(blob) - 1):
        bad = bytearray(blob)
        bad[pos] ^= 0x80
        with pytest.raises(DecryptionError):
            g.decrypt(bytes(bad), key)
    with pytest.raises(DecryptionError):
        g.decrypt(blob[:27], key)  # shorter than nonce + tag
    with pytest.raises(DecryptionError):
        g.decrypt(blob, rnd.randbytes(32))
    # a 16-byte key through a 256-bit adapter works, as AESGCM(key) does
    k16 = rnd.randbytes(16)
    assert g.decrypt(g.encrypt(data, k16), k16) == data


def test_device_buffers_unaligned(oracle):
    """Device entry points with inputs and outputs off 4-byte alignment (the byte path) and on
    it, and decrypt verdicts per blob."""
    rnd = random.Random(3)
    g = GpuAesGcm()
    hs = torch.cuda.current_stream().cuda_stream
    lens = [100_001, 16, 0, 70_000, 5]
    datas = [rnd.randbytes(n) for n in lens]
    keys = [rnd.randbytes(32) for _ in lens]
    nonces = [rnd.randbytes(12) for _ in lens]
    shifts = [1, 2, 3, 0, 1]
    ins = [dev(bytes(s) + d) for s, d in zip(shifts, datas)]
    kt, nt = dev(b''.join(keys)), dev(b''.join(nonces))
    outs = [torch.zeros(3 + 12 + n + 16, dtype=torch.uint8, device='cuda') for n in lens]
    g.encrypt_device([t.data_ptr() + s for t, s in zip(ins, shifts)], lens,
                     [kt.data_ptr() + 32 * i for i in range(len(lens))],
                     [nt.data_ptr() + 12 * i for i in range(len(lens))],
                     [o.data_ptr() + 3 for o in outs], hs)
    torch.cuda.synchronize()
    blobs = [o.cpu().numpy()[3:].tobytes() for o in outs]
    for d, k, v, b in zip(datas, keys, nonces, blobs):
        assert b == v + oracle.gcm_encrypt(k, v, d)
    blobs[3] = blobs[3][:40] + bytes([blobs[3][40] ^ 1]) + blobs[3][41:]
    bins = [dev(b) for b in blobs]
    pouts = [torch.zeros(max(n, 1), dtype=torch.uint8, device='cuda') for n in lens]
    ok = torch.zeros(len(lens), dtype=torch.uint8, device='cuda')
    g.decrypt_device([t.data_ptr() for t in bins], [len(b) for b in blobs],
                     [kt.data_ptr() + 32 * i for i in range(len(lens))],
                     [p.data_ptr() for p in pouts], ok.data_ptr(), hs)
    torch.cuda.synchronize()
    assert ok.cpu().tolist() == [1, 1, 1, 0, 1]
    for i in (0, 1, 4):
        assert pouts[i].cpu().numpy()[:lens[i]].tobytes() == datas[i]


def test_many_small_messages(oracle):
    """Thousands of short items through the work counter."""
    rnd = random.Random(4)
    n = 3000
    datas = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(n)]
    keys = [rnd.randbytes(24) for _ in range(n)]
    nonces = [rnd.randbytes(12) for _ in range(n)]
    g = GpuAesGcm(key_bits=192)
    blobs = g.encrypt_many(datas, keys, nonces)
    for i in range(0, n, 97):
        assert blobs[i] == nonces[i] + oracle.gcm_encrypt(keys[i], nonces[i], datas[i])
    assert g.decrypt_many(blobs, keys) == datas


@pytest.mark.parametrize('key_bits', [256, 128])
def test_chunk_path(oracle, key_bits):
    """chunk -> digest -> derive_shared_subkey -> encrypt, all in HBM (repository.py:1454-1473),
    against hashlib (digest, subkey) and the oracle (every blob)."""
    rnd = random.Random(key_bits)
    mn, mx = 2_000, 80_000
    lens = [(3 << 20) - 7 * i for i in range(4)] + [0, 999]
    datas = [rnd.randbytes(n) for n in lens]
    ch = GpuChunker(mn, mx, synth.seeded_key(11))
    h = GpuBlake2b(length=64)
    g = GpuAesGcm(key_bits=key_bits)
    hs = torch.cuda.current_stream().cuda_stream
    ts = [dev(d) for d in datas]
    ptrs = [t.data_ptr() for t in ts]
    total, caps = ch.capacity(lens)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(len(lens), dtype=torch.int64, device='cuda')
    dig = torch.zeros((total, SLOT), dtype=torch.uint8, device='cuda')
    keys = torch.zeros((total, SLOT), dtype=torch.uint8, device='cuda')
    nonces_h = os.urandom(total * 12)
    nonces = dev(nonces_h)
    shared, salt = rnd.randbytes(32), rnd.randbytes(16)
    kdf = dev(state_init(g.key_bytes, key=shared, salt=salt))
    out_total, base = g.chunks_layout(ch, lens)
    out = torch.zeros(out_total, dtype=torch.uint8, device='cuda')
    ch.chunk_device(ptrs, lens, None, cuts.data_ptr(), counts.data_ptr(), hs)
    h.digest_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), dig.data_ptr(), hs)
    h.derive_chunks(ch, lens, counts.data_ptr(), kdf.data_ptr(), dig.data_ptr(), keys.data_ptr(), hs)
    g.encrypt_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), keys.data_ptr(),
                     nonces.data_ptr(), out.data_ptr(), hs)
    torch.cuda.synchronize()
    cuts_h = cuts.cpu().numpy().view(np.uint64)
    counts_h = counts.cpu().numpy()
    dig_h, keys_h, out_h = dig.cpu().numpy(), keys.cpu().numpy(), out.cpu().numpy()
    cbase = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    seen = 0
    for i, data in enumerate(datas):
        ends = [int(e) for e in cuts_h[cbase[i]:cbase[i] + counts_h[i]]]
        assert ends == oracle.chunk_stream(data, mn, mx, synth.seeded_key(11), 0)
        s = 0
        for k, e in enumerate(ends):
            slot = int(cbase[i]) + k
            chunk = data[s:e]
            d = hashlib.blake2b(chunk).digest()
            assert dig_h[slot].tobytes() == d
            sk = hashlib.blake2b(d, salt=salt, key=shared, digest_size=g.key_bytes).digest()
            assert keys_h[slot, :g.key_bytes].tobytes() == sk
            o = int(base[i]) + s + k * 28
            blob = out_h[o:o + 28 + len(chunk)].tobytes()
            v = nonces_h[12 * slot:12 * slot + 12]
            assert blob == v + oracle.gcm_encrypt(sk, v, chunk), (i, k)
            s = e
            seen += 1
    assert seen == int(counts_h.sum()) > 100
