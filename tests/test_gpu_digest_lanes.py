"""The one-lane-per-chunk form of the BLAKE2b digest kernel (blake2b.hip lane_hash): the same
hashlib checks as tests/test_gpu_digest.py with the lane / quad split forced through
RC_B2_LANE_MAX (read per call): every item by lanes, a mixed split, and the default split on a
batch of many short chunks (config 3 iii's parameters), where most chunks take lanes.  Kernel
ids: rc_b2_kernel's lane role, blake2b.hip lane_hash."""

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import test_gpu_digest as D  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402
from replicat_amd.hashing import GpuBlake2b  # noqa: E402

SPLITS = {'all_lanes': str(1 << 40), 'mixed': '3000'}


@pytest.fixture(params=sorted(SPLITS))
def split(request, monkeypatch):
    monkeypatch.setenv('RC_B2_LANE_MAX', SPLITS[request.param])
    return request.param


@pytest.fixture(scope='module')
def hasher():
    return GpuBlake2b(length=64)


def test_block_boundaries_lanes(split, hasher):
    D.test_block_boundaries(hasher)


@pytest.mark.parametrize('size', [1, 20, 33, 64])
def test_digest_sizes_lanes(split, size):
    D.test_digest_sizes(size)


def test_many_random_lengths_lanes(split, hasher):
    D.test_many_random_lengths(hasher)


def test_unaligned_device_buffers_lanes(split, hasher):
    D.test_unaligned_device_buffers(hasher)


def test_buffer_ending_at_allocation_end_lanes(split, hasher):
    D.test_buffer_ending_at_allocation_end(hasher)


@pytest.mark.parametrize('mn,mx', [(2_000, 80_000), (4, 64), (60, 200)])
def test_chunk_digests_lanes(split, hasher, mn, mx):
    D.test_chunk_digests_match_hashlib(hasher, mn, mx)


def test_many_short_chunks_default_split(hasher, monkeypatch):
    """8192 x 1 MiB streams at min 2,000 / max 80,000: 8 GiB is throughput-bound (>= 80,000 << 16
    bytes), so the default split sends chunks of up to 64 KiB to lanes and the rest to quads;
    every chunk of a sample of streams = hashlib."""
    monkeypatch.delenv('RC_B2_LANE_MAX', raising=False)
    n, size = 8192, 1 << 20
    ch = GpuChunker(2_000, 80_000, b'\xff' * 16)
    ts, res = D._chunk_and_digest(ch, hasher, [size] * n)
    short = 0
    for i in list(range(0, n, 193)) + [n - 1]:
        data = synth.stream_bytes(size, synth.DEFAULT_SEED, i).tobytes()
        ends, dig = res[i]
        prev = 0
        for k, e in enumerate(ends):
            assert dig[k].tobytes() == D.H(data[prev:e]), (i, k)
            short += (e - prev) <= (n * size) >> 17
            prev = e
    assert short > 0  # the sample includes lane-hashed chunks
    del ts
    torch.cuda.empty_cache()
