"""GPU parity of the BLAKE2b chunk digests (replicat_amd/csrc/blake2b.hip through the C ABI of
include/replicat_digest.h) against hashlib -- the implementation replicat's `blake2b.digest`
calls (replicat/utils/adapters.py:224-225) -- and the oracle's RFC 7693 restatement.
Bit-exact.  Runs on an MI355X only (-m gpu)."""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from gpu_util import chunk_device, device_streams  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402
from replicat_amd.hashing import SLOT, GpuBlake2b, chunk_digest_host  # noqa: E402


def H(data, size=64):
    return hashlib.blake2b(bytes(data), digest_size=size).digest()


def cur_stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope='module')
def hasher():
    return GpuBlake2b(length=64)


def test_rfc7693_abc(hasher):
    assert hasher.digest(b'abc').hex().startswith('ba80a53f981c4d0d')


def test_block_boundaries(hasher):
    rnd = random.Random(1)
    msgs = [rnd.randbytes(n) for n in list(range(0, 300)) + [383, 384, 385, 1023, 1024, 1025]]
    assert hasher.digest_many(msgs) == [H(m) for m in msgs]


@pytest.mark.parametrize('size', [1, 7, 20, 32, 48, 63, 64])
def test_digest_sizes(size):
    h = GpuBlake2b(length=size)
    rnd = random.Random(size)
    msgs = [rnd.randbytes(rnd.randrange(0, 3000)) for _ in range(70)]
    assert h.digest_many(msgs) == [H(m, size) for m in msgs]


def test_many_random_lengths(hasher):
    rnd = random.Random(5)
    msgs = [rnd.randbytes(rnd.choice([rnd.randrange(0, 600), rnd.randrange(0, 200_000),
                                      rnd.randrange(1 << 20, 3 << 20)])) for _ in range(300)]
    assert hasher.digest_many(msgs) == [H(m) for m in msgs]


def test_unaligned_device_buffers(hasher):
    """Any start alignment (a stream's tail chunk starts anywhere) and any length."""
    rnd = random.Random(9)
    raw = rnd.randbytes(1 << 20)
    t = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device='cuda')
    ptrs, lens, exp = [], [], []
    for off in range(0, 64):
        for n in (0, 1, 3, 5, 127, 128, 129, 255, 256, 1000, rnd.randrange(0, 100_000)):
            ptrs.append(t.data_ptr() + off)
            lens.append(n)
            exp.append(H(raw[off:off + n]))
    out = torch.zeros((len(ptrs), SLOT), dtype=torch.uint8, device='cuda')
    hasher.digest_device(ptrs, lens, out.data_ptr(), cur_stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert [got[i].tobytes() for i in range(len(exp))] == exp


def test_buffer_ending_at_allocation_end(hasher):
    """Messages whose last byte is the last byte of their allocation, every tail alignment:
    the kernel never reads past a message's last dword."""
    rnd = random.Random(4)
    for n in (1, 2, 3, 4, 5, 127, 129, 4093, 4097, 65_535):
        raw = rnd.randbytes(n)
        t = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device='cuda')
        out = torch.zeros(SLOT, dtype=torch.uint8, device='cuda')
        hasher.digest_device([t.data_ptr()], [n], out.data_ptr(), cur_stream())
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == H(raw)


def _chunk_and_digest(ch, hasher, sizes, last=None, ids=None, seed=synth.DEFAULT_SEED):
    ts = device_streams(sizes, seed=seed, ids=ids)
    total, caps = ch.capacity(sizes)
    cuts = torch.zeros(max(total, 1), dtype=torch.int64, device='cuda')
    counts = torch.zeros(len(sizes), dtype=torch.int64, device='cuda')
    dig = torch.zeros((max(total, 1), SLOT), dtype=torch.uint8, device='cuda')
    ptrs = [t.data_ptr() for t in ts]
    ch.chunk_device(ptrs, sizes, last, cuts.data_ptr(), counts.data_ptr(), cur_stream())
    hasher.digest_chunks(ch, ptrs, sizes, cuts.data_ptr(), counts.data_ptr(), dig.data_ptr(),
                         cur_stream())
    torch.cuda.synchronize()
    cuts_h = cuts.cpu().numpy().view(np.uint64)
    counts_h = counts.cpu().numpy()
    dig_h = dig.cpu().numpy()
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    return ts, [(cuts_h[b:b + c].tolist(), dig_h[b:b + c]) for b, c in zip(base, counts_h)]


@pytest.mark.parametrize('mn,mx', [(2_000, 80_000), (128_000, 5_120_000), (4, 64), (60, 200)])
def test_chunk_digests_match_hashlib(hasher, mn, mx):
    rnd = random.Random(mn)
    sizes = [0, 1, 5, 4096, 3 * mx + 7, 2 * mx - 1] + [rnd.randrange(0, 6 * mx) for _ in range(12)]
    sizes = [min(s, 24 << 20) for s in sizes]
    last = [rnd.randrange(0, s + 1) for s in sizes]
    ch = GpuChunker(mn, mx, synth.seeded_key(mn))
    ts, res = _chunk_and_digest(ch, hasher, sizes, last)
    for i, (n, (ends, dig)) in enumerate(zip(sizes, res)):
        data = synth.stream_bytes(n, synth.DEFAULT_SEED, i).tobytes()
        assert (ends[-1] if ends else 0) == n
        prev = 0
        for k, e in enumerate(ends):
            assert dig[k].tobytes() == H(data[prev:e]), (i, k, prev, e)
            prev = e


def test_chunk_digests_config2_sample(hasher):
    """16 of config 2's 64 MiB streams (default parameters, key ff): every chunk's digest."""
    ids = [0, 1, 2, 3, 100, 255, 256, 511, 512, 700, 800, 900, 1000, 1021, 1022, 1023]
    sizes = [64 << 20] * len(ids)
    ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
    ts, res = _chunk_and_digest(ch, hasher, sizes, ids=ids)
    for sid, n, (ends, dig) in zip(ids, sizes, res):
        data = synth.stream_bytes(n, synth.DEFAULT_SEED, sid).tobytes()
        prev = 0
        for k, e in enumerate(ends):
            assert dig[k].tobytes() == H(data[prev:e]), (sid, k)
            prev = e


def test_chunk_digest_host_path(hasher, oracle):
    """rc_chunk_digest_host (pinned copies in, cuts + digests out) = oracle cuts + hashlib."""
    rnd = random.Random(12)
    mn, mx = 2_000, 80_000
    key = synth.seeded_key(12)
    ch = GpuChunker(mn, mx, key)
    bufs = [np.frombuffer(rnd.randbytes(rnd.randrange(0, 3 << 20)), dtype=np.uint8)
            for _ in range(9)]
    last = [rnd.randrange(0, b.size + 1) for b in bufs]
    ends, digs = chunk_digest_host(ch, hasher, bufs, last)
    for b, P, e, d in zip(bufs, last, ends, digs):
        exp = oracle.chunk_stream(b, mn, mx, key, P)
        assert e.tolist() == exp
        prev = 0
        for k, x in enumerate(exp):
            assert d[k].tobytes() == H(b[prev:x].tobytes())
            prev = x


def test_digest_matches_oracle_restatement(hasher, oracle):
    rnd = random.Random(21)
    msgs = [rnd.randbytes(rnd.randrange(0, 50_000)) for _ in range(40)]
    assert hasher.digest_many(msgs) == [oracle.blake2b(m) for m in msgs]
