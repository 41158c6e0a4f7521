"""The one-lane-per-chunk form of the BLAKE2b digests (blake2b.hip lane_hash): the same hashlib
checks as tests/test_gpu_digest.py with the lane / quad split forced through RC_B2_LANE_MAX and
RC_B2_LANE_ONLY (read when the hasher is created): every item by the lane kernel (rc_b2_lane_kernel), every item by
the fused kernel's lane role (rc_b2_kernel), a mixed split, and the default split on batches of
many short chunks (config 3 iii's parameters): a mixed one and a lane-only one."""

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import test_gpu_digest as D  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402
from replicat_amd.hashing import GpuBlake2b  # noqa: E402

# (RC_B2_LANE_MAX, RC_B2_LANE_ONLY): every item by the lane kernel; every item by the fused
# kernel's lane role; the fused kernel with quads above 3,000 bytes and lanes below
SPLITS = {'all_lanes': (str(1 << 40), '1'), 'all_lanes_fused': (str(1 << 40), '0'),
          'mixed': ('3000', '1')}


@pytest.fixture(params=sorted(SPLITS))
def split(request, monkeypatch):
    lane_max, lane_only = SPLITS[request.param]
    monkeypatch.setenv('RC_B2_LANE_MAX', lane_max)
    monkeypatch.setenv('RC_B2_LANE_ONLY', lane_only)
    return request.param


@pytest.fixture
def hasher(split):
    # the split knobs are read when a hasher is created (knobs.h): one per setting
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


@pytest.mark.parametrize('n', [8192, 16384])
def test_many_short_chunks_default_split(monkeypatch, n):
    """n x 1 MiB streams at min 2,000 / max 80,000, throughput-bound (>= 80,000 << 16 bytes): at
    8 GiB the default split sends chunks of up to 64 KiB to lanes and the rest to quads (the
    fused kernel); at 16 GiB every chunk fits a lane (up to 128 KiB: the lane kernel).  Every
    chunk of a sample of streams = hashlib."""
    monkeypatch.delenv('RC_B2_LANE_MAX', raising=False)
    monkeypatch.delenv('RC_B2_LANE_ONLY', raising=False)
    hasher = GpuBlake2b(length=64)  # the default split (knobs read at creation)
    size = 1 << 20
    ch = GpuChunker(2_000, 80_000, b'\xff' * 16)
    ts, res = D._chunk_and_digest(ch, hasher, [size] * n)
    short = 0
    for i in list(range(0, n, n // 40 + 1)) + [n - 1]:
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
