"""GPU parity of the incremental and keyed BLAKE2b (rc_blake2b_update_device, blake2b.hip
rc_b2_update_kernel) against hashlib -- what replicat's blake2b adapter calls for
`incremental_hasher()` (replicat/utils/adapters.py:106-114,227-228; the per-file digest of
replicat/repository.py:1433-1446), `derive` (adapters.py:203-211: the shared-subkey KDF of
encrypted repositories, repository.py:132-137) and `mac` (adapters.py:217-221).  Bit-exact.
Runs on an MI355X only (-m gpu)."""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from replicat_amd.hashing import (SLOT, STATE_BYTES, DeviceIncrementalHasher,  # noqa: E402
                                  GpuBlake2b, state_init)


def cur_stream():
    return torch.cuda.current_stream().cuda_stream


def dev_bytes(data, offset=0):
    """Device copy of data starting `offset` bytes into a fresh allocation (misalignment)."""
    t = torch.zeros(len(data) + offset + 16, dtype=torch.uint8, device='cuda')
    if len(data):
        t[offset:offset + len(data)].copy_(torch.from_numpy(np.frombuffer(bytes(data), np.uint8).copy()))
    return t, t.data_ptr() + offset


def dev_states(records):
    t = torch.from_numpy(np.frombuffer(b''.join(records), np.uint8).copy()).cuda()
    return t, [t.data_ptr() + STATE_BYTES * i for i in range(len(records))]


@pytest.fixture(scope='module')
def h64():
    return GpuBlake2b(length=64)


@pytest.mark.parametrize('splits', [
    [], [0], [1], [127], [128], [129], [128, 128], [127, 1], [1, 127, 1], [0, 0, 5],
    [256, 0, 128], [1000, 3, 128 * 7, 129], [200_000, 77, 1 << 20]])
def test_incremental_splits(h64, splits):
    rnd = random.Random(len(splits) * 7919 + sum(splits))
    inc = DeviceIncrementalHasher(h64)
    ref = hashlib.blake2b(digest_size=64)
    for n in splits:
        piece = rnd.randbytes(n)
        inc.feed(piece)
        ref.update(piece)
    assert inc.digest() == ref.digest()


@pytest.mark.parametrize('size', [1, 20, 32, 64])
def test_incremental_digest_sizes(size):
    h = GpuBlake2b(length=size)
    rnd = random.Random(size)
    inc = DeviceIncrementalHasher(h)
    ref = hashlib.blake2b(digest_size=size)
    for _ in range(6):
        piece = rnd.randbytes(rnd.randrange(0, 5000))
        inc.feed(piece)
        ref.update(piece)
    assert inc.digest() == ref.digest()


@pytest.mark.parametrize('klen', [0, 1, 16, 32, 63, 64])
@pytest.mark.parametrize('mlen', [0, 1, 64, 127, 128, 129, 4096, 70_001])
def test_keyed_salted(h64, klen, mlen):
    rnd = random.Random(klen * 1000 + mlen)
    key, salt, person = rnd.randbytes(klen), rnd.randbytes(rnd.randrange(0, 17)), rnd.randbytes(rnd.randrange(0, 17))
    msg = rnd.randbytes(mlen)
    size = rnd.choice([16, 32, 64])
    st, (sp,) = dev_states([state_init(size, key=key, salt=salt, person=person)])
    buf, p = dev_bytes(msg, offset=rnd.randrange(4))
    out = torch.zeros(SLOT, dtype=torch.uint8, device='cuda')
    h64.update_device([sp], [p], [mlen], [1], out.data_ptr(), cur_stream())
    torch.cuda.synchronize()
    exp = hashlib.blake2b(msg, digest_size=size, key=key, salt=salt, person=person).digest()
    got = out.cpu().numpy().tobytes()
    assert got[:size] == exp and got[size:] == bytes(SLOT - size)


def test_kdf_shared_state(h64):
    """adapters.py:203-211: derive(key_material, params=salt, context=digest) for many chunk
    digests through ONE read-only device state (the shared key never changes per call)."""
    rnd = random.Random(11)
    shared_key, salt = rnd.randbytes(64), rnd.randbytes(16)
    contexts = [rnd.randbytes(64) for _ in range(3000)]
    st, (sp,) = dev_states([state_init(32, key=shared_key, salt=salt)])
    ctx, base = dev_bytes(b''.join(contexts))
    out = torch.zeros((len(contexts), SLOT), dtype=torch.uint8, device='cuda')
    n = len(contexts)
    h64.update_device([sp] * n, [base + 64 * i for i in range(n)], [64] * n, [1] * n,
                      out.data_ptr(), cur_stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i, c in enumerate(contexts):
        exp = hashlib.blake2b(c, salt=salt, digest_size=32, key=shared_key).digest()
        assert got[i, :32].tobytes() == exp, i
    # the state was left untouched by the final items
    assert st.cpu().numpy().tobytes() == state_init(32, key=shared_key, salt=salt)


def test_batched_files_across_batches(h64):
    """Per-file digests of files fed in several device calls (one state per file, mixed
    final / non-final items per call, misaligned buffers): the snapshot's _stream_files
    incremental hasher (repository.py:1433-1446) over batch boundaries."""
    rnd = random.Random(3)
    nfiles = 200
    files = [rnd.randbytes(rnd.choice([0, 1, 127, 128, 129, rnd.randrange(0, 3000),
                                       rnd.randrange(0, 400_000)])) for _ in range(nfiles)]
    st, sps = dev_states([state_init(64)] * nfiles)
    pos = [0] * nfiles
    done = [False] * nfiles
    out = torch.zeros((nfiles, SLOT), dtype=torch.uint8, device='cuda')
    while not all(done):
        idx, ptrs, lens, fin, keep = [], [], [], [], []
        for i in range(nfiles):
            if done[i]:
                continue
            left = len(files[i]) - pos[i]
            take = min(left, rnd.choice([0, 1, 100, 128, 129, 5000, 1 << 17]))
            last = take == left and rnd.random() < 0.7
            buf, p = dev_bytes(files[i][pos[i]:pos[i] + take], offset=rnd.randrange(4))
            keep.append(buf)
            idx.append(i)
            ptrs.append(p)
            lens.append(take)
            fin.append(1 if last else 0)
            pos[i] += take
            done[i] = last
        # final digests land in slot j of this call: scatter them through a scratch output
        scratch = torch.zeros((len(idx), SLOT), dtype=torch.uint8, device='cuda')
        h64.update_device([sps[i] for i in idx], ptrs, lens, fin, scratch.data_ptr(), cur_stream())
        torch.cuda.synchronize()
        for j, i in enumerate(idx):
            if fin[j]:
                out[i].copy_(scratch[j])
    got = out.cpu().numpy()
    for i, f in enumerate(files):
        assert got[i].tobytes() == hashlib.blake2b(f).digest(), i


def test_mac_of_digests(h64):
    """adapters.py:217-221: mac(message, params=key) = blake2b(message, key=params)."""
    rnd = random.Random(5)
    key = rnd.randbytes(64)
    msgs = [rnd.randbytes(64) for _ in range(500)]
    st, (sp,) = dev_states([state_init(64, key=key)])
    buf, base = dev_bytes(b''.join(msgs))
    out = torch.zeros((len(msgs), SLOT), dtype=torch.uint8, device='cuda')
    h64.update_device([sp] * len(msgs), [base + 64 * i for i in range(len(msgs))],
                      [64] * len(msgs), [1] * len(msgs), out.data_ptr(), cur_stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i, m in enumerate(msgs):
        assert got[i].tobytes() == hashlib.blake2b(m, key=key).digest()
