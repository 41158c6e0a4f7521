"""Time the encrypted-snapshot device leg on config 2 (1024 x 64 MiB, default params).

Chunk once, then per repetition: BLAKE2b-512 digest of every chunk (repository.py:1462), its
subkey derive_shared_subkey(digest) (keyed BLAKE2b-256, :1470-1472) and its AES-256-GCM
encryption (:1470-1473), each stage bracketed by HIP events on the launch stream.  A sample of
chunks is checked end to end: digest against hashlib, subkey against hashlib.blake2b(digest,
salt=, key=), and the blob decrypted (on the device) back to the chunk.  The CPU reference for the
cipher is OpenSSL's EVP AES-256-GCM (what `cryptography`'s AESGCM binds), timed on one host core.

    python scripts/gcm_probe.py [streams] [stream_mib] [min] [max]
"""
import hashlib
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix  # noqa: E402
from replicat_amd.cipher import GpuAesGcm  # noqa: E402
from replicat_amd.hashing import SLOT, GpuBlake2b, state_init  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 128_000
mx = int(sys.argv[4]) if len(sys.argv) > 4 else 5_120_000
reps = 3
size = mib << 20
GIB = float(1 << 30)

torch.cuda.set_device(0)
hs = torch.cuda.current_stream().cuda_stream
pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
ptrs = [pool.data_ptr() + i * size for i in range(n)]
for i, p in enumerate(ptrs):
    fill_splitmix(p, size, synth.DEFAULT_SEED, i, hs)
lens = [size] * n
ch = GpuChunker(mn, mx, b'\xff' * 16)
h = GpuBlake2b(length=64)
g = GpuAesGcm(key_bits=256, nonce_bits=96)
total, caps = ch.capacity(lens)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
dig = torch.zeros((total, SLOT), dtype=torch.uint8, device='cuda')
keys = torch.zeros((total, SLOT), dtype=torch.uint8, device='cuda')
nonces_h = os.urandom(total * 12)
nonces = torch.from_numpy(np.frombuffer(nonces_h, dtype=np.uint8).copy()).cuda()
shared, salt = os.urandom(32), os.urandom(16)
kdf = torch.from_numpy(np.frombuffer(state_init(32, key=shared, salt=salt), np.uint8).copy()).cuda()
out_total, base = g.chunks_layout(ch, lens)
out = torch.empty(out_total, dtype=torch.uint8, device='cuda')
ch.chunk_device(ptrs, lens, None, cuts.data_ptr(), counts.data_ptr(), hs)
torch.cuda.synchronize()
nchunks = int(counts.sum().item())


def digest():
    h.digest_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), dig.data_ptr(), hs)


def derive():
    h.derive_chunks(ch, lens, counts.data_ptr(), kdf.data_ptr(), dig.data_ptr(), keys.data_ptr(), hs)


def encrypt():
    g.encrypt_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), keys.data_ptr(),
                     nonces.data_ptr(), out.data_ptr(), hs)


stages = (('digest', digest), ('derive', derive), ('encrypt', encrypt))
for _, fn in stages:  # warm-up
    fn()
torch.cuda.synchronize()
ms = {name: 0.0 for name, _ in stages}
for _ in range(reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 1)]
    ev[0].record()
    for k, (_, fn) in enumerate(stages):
        fn()
        ev[k + 1].record()
    torch.cuda.synchronize()
    for k, (name, _) in enumerate(stages):
        ms[name] += ev[k].elapsed_time(ev[k + 1]) / reps
print(json.dumps({'progress': 'timed', 'ms': ms}), flush=True)

# end-to-end check on a sample of chunks
cuts_h = cuts.cpu().numpy().view(np.uint64)
counts_h = counts.cpu().numpy()
cbase = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
rnd = random.Random(1)
checked = 0
for i in rnd.sample(range(n), min(n, 8)):
    ends = [0] + [int(e) for e in cuts_h[cbase[i]:cbase[i] + counts_h[i]]]
    data = pool[i * size:(i + 1) * size].cpu().numpy()
    for k in rnd.sample(range(len(ends) - 1), min(len(ends) - 1, 2)):
        s, e = ends[k], ends[k + 1]
        slot = int(cbase[i]) + k
        chunk = data[s:e].tobytes()
        d = hashlib.blake2b(chunk).digest()
        assert dig[slot].cpu().numpy().tobytes() == d, (i, k)
        sk = hashlib.blake2b(d, salt=salt, key=shared, digest_size=32).digest()
        assert keys[slot, :32].cpu().numpy().tobytes() == sk, (i, k)
        o = int(base[i]) + s + 28 * k
        blob = out[o:o + 28 + (e - s)].cpu().numpy().tobytes()
        assert blob[:12] == nonces_h[12 * slot:12 * slot + 12]
        assert g.decrypt(blob, sk) == chunk, (i, k)
        checked += 1

# CPU reference: OpenSSL EVP AES-256-GCM on one host core (tests/golden/make_gcm_golden.py)
cpu = None
try:
    sys.path.insert(0, os.path.join('tests', 'golden'))
    from make_gcm_golden import openssl_gcm_encrypt  # noqa: E402
    blk = os.urandom(64 << 20)
    openssl_gcm_encrypt(bytes(32), bytes(12), blk[:1 << 20])
    t0 = time.perf_counter()
    for _ in range(4):
        openssl_gcm_encrypt(os.urandom(32), os.urandom(12), blk)
    cpu = round(4 * len(blk) / (time.perf_counter() - t0) / GIB, 2)
except Exception as exc:  # no libcrypto on the host: report why
    cpu = f'unavailable: {exc}'

nbytes = n * size
print(json.dumps({'streams': n, 'stream_mib': mib, 'min': mn, 'max': mx, 'chunks': nchunks,
                  'digest_ms': round(ms['digest'], 3), 'derive_ms': round(ms['derive'], 3),
                  'encrypt_ms': round(ms['encrypt'], 3),
                  'digest_gib_s': round(nbytes / (ms['digest'] * 1e-3) / GIB, 1),
                  'encrypt_gib_s': round(nbytes / (ms['encrypt'] * 1e-3) / GIB, 1),
                  'encrypt_gb_s': round(nbytes / (ms['encrypt'] * 1e-3) / 1e9, 1),
                  'digest_derive_encrypt_gib_s': round(nbytes / (sum(ms.values()) * 1e-3) / GIB, 1),
                  'sample_checked': checked,
                  'cpu_openssl_aes256gcm_gib_s_1core': cpu}), flush=True)
