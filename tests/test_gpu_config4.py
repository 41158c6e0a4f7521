"""GPU parity at BASELINE config 4 (SURVEY.md §8 d): 128 streams x 8 GiB, stream i on GPU i mod 8.

tests/golden/config4.json holds the REFERENCE's cut lists (make_golden.py --config4: its own
``next_cut``, compiled from /root/reference/src/adapters.cpp, over every 8 GiB stream, and its
adapter over 16 MiB pieces for stream 0) as per-stream SHA-256 digests plus, per GPU, the digest
over that GPU's 16 streams in shard order.  Here one MI355X holds a whole GPU's shard -- 16 x
8 GiB = 128 GiB resident -- and chunks it in ONE rc_chunk_device call: 64-bit offsets past 4 GiB,
and every stream's argmax region split into ~50 chain segments that run together.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import bench  # noqa: E402

from replicat_amd.chunker import GpuChunker, fill_splitmix  # noqa: E402

C4 = G.load('config4.json')
PER_STREAM = {s['id']: s for s in C4['per_stream']}


def _hs():
    return torch.cuda.current_stream().cuda_stream


def _chunk_shard(gpu, n_streams=16):
    ids = bench.shard_ids('4', gpu, n_streams)
    size = C4['size']
    ch = GpuChunker(C4['min'], C4['max'], b'\xff' * 16)
    slot = size + 64
    pool = torch.empty(n_streams * slot + 64, dtype=torch.uint8, device='cuda')
    ptrs = [pool.data_ptr() + k * slot for k in range(n_streams)]
    for p, i in zip(ptrs, ids):
        fill_splitmix(p, size, C4['seed'], i, _hs())
    lens = [size] * n_streams
    total, caps = ch.capacity(lens)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n_streams, dtype=torch.int64, device='cuda')
    ch.chunk_device(ptrs, lens, None, cuts.data_ptr(), counts.data_ptr(), _hs())
    _, _, ends = bench.cut_digest(cuts, counts, caps)
    del pool, cuts, counts
    torch.cuda.empty_cache()
    return ids, ends


@pytest.mark.parametrize('gpu', [0, 5])
def test_config4_shard_matches_reference(gpu):
    """A whole GPU's shard (16 x 8 GiB) in one call: every stream's cut list and the shard's
    digest equal the reference's."""
    ids, ends = _chunk_shard(gpu)
    g = C4['per_gpu'][gpu]
    assert ids == g['ids']
    for i, e in zip(ids, ends):
        s = PER_STREAM[i]
        lst = e.tolist()
        assert lst[:8] == s['first_ends'] and lst[-8:] == s['last_ends'], i
        assert len(lst) == s['chunks'] and G.cutlist_digest([e]) == s['sha256'], i
        assert lst[-1] == C4['size']
    assert G.cutlist_digest(ends) == g['sha256']
    assert sum(len(e) for e in ends) == g['chunks']


def test_config4_offsets_past_32_bits():
    """The cut offsets of an 8 GiB stream pass 2**32 and stay strictly increasing."""
    ids, ends = _chunk_shard(1, n_streams=2)
    for i, e in zip(ids, ends):
        assert int(e[-1]) == C4['size'] > 1 << 32
        assert np.all(np.diff(e.astype(np.int64)) > 0)
        assert G.cutlist_digest([e]) == PER_STREAM[i]['sha256']
