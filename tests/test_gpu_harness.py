"""GPU parity for the remaining BASELINE workloads whose checks lived only in bench lines:

* the reference's own benchmark stream (Repository._benchmark_chunker,
  /root/reference/replicat/repository.py:1984-2008): 10 x 512,000,000 Random(0) bytes fed to
  the adapter as 10 pieces, i.e. ONE stream of 5.12 GB whose last piece starts at L - 512 MB.
  tests/golden/harness.json holds the reference adapter's 1,728 cuts of it (count, SHA-256,
  first and last ends; make_golden.py ran replicat's adapter over the reference extension);
* config 3 (i) at full size: 65,536 x 1 MiB streams, default parameters.  Every stream is
  shorter than max_length, so the reference's next_cut emits it whole by the tail rule
  (src/adapters.cpp:50-51: size <= max -> size): one cut per stream, at L;
* config 2 with an encrypted repository's key (repository.py:174-181 chooses
  key.params['chunker_params']): the first 128 streams against the reference's digest, as
  bench.py's seeded-key line now checks.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from gpu_util import chunk_device  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import (MAX_LENGTH, MIN_LENGTH, GpuChunker,  # noqa: E402
                                  fill_splitmix_streams)

MIB = 1 << 20


def _hs():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize('seg', [None, (5_120_000, 1), (2 * 5_120_000, 0)])
def test_reference_harness_stream(seg, monkeypatch):
    """seg = (segment bytes, extension steps) forced: one-max segments with one extension step
    (most boundaries repaired by the merge kernel), two-max segments with none."""
    if seg is not None:
        monkeypatch.setenv('RC_SEGMENT_BYTES', str(seg[0]))
        monkeypatch.setenv('RC_SEGMENT_EXT', str(seg[1]))
    g = G.load('harness.json')
    assert (g['min'], g['max'], g['params']) == (MIN_LENGTH, MAX_LENGTH, None)
    L = g['length']
    dev = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for piece in synth.harness_buffers(g['number'], g['size'], g['seed']):
        dev[off:off + len(piece)].copy_(torch.frombuffer(piece, dtype=torch.uint8))
        off += len(piece)
    assert off == L
    ch = GpuChunker(g['min'], g['max'], b'\xff' * 16)
    ends = chunk_device(ch, [dev], [L], [g['last_piece']])[0]
    assert len(ends) == g['chunks']
    assert ends[:len(g['first_ends'])] == g['first_ends']
    assert ends[-len(g['last_ends']):] == g['last_ends']
    assert G.cutlist_digest([ends]) == g['sha256']
    del dev
    torch.cuda.empty_cache()


def test_config3i_full_size():
    """65,536 x 1 MiB, defaults, one piece per stream: one chunk of L bytes per stream."""
    n, size = 65536, MIB
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, _hs())
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    total, caps = ch.capacity([size] * n)
    cuts = torch.full((total,), -1, dtype=torch.int64, device='cuda')
    counts = torch.full((n,), -1, dtype=torch.int64, device='cuda')
    base = pool.data_ptr()
    ch.chunk_device(np.arange(n, dtype=np.uint64) * size + base, [size] * n, None,
                    cuts.data_ptr(), counts.data_ptr(), _hs())
    torch.cuda.synchronize()
    counts_h = counts.cpu().numpy()
    assert (counts_h == 1).all()
    starts = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    first = cuts.cpu().numpy()[starts]
    assert (first == size).all()
    del pool, cuts
    torch.cuda.empty_cache()


def test_config2_seeded_key_first128():
    g = {d['name']: d for d in G.load('digests.json')}['config2_seeded_first128']
    key = bytes.fromhex(g['params'])
    assert key == synth.seeded_key(1)
    n, size = g['streams'], g['size']
    slot = size
    pool = torch.empty(n * slot + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, slot, g['seed'], 0, 1, _hs())
    ch = GpuChunker(g['min'], g['max'], key)
    total, caps = ch.capacity([size] * n)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    ch.chunk_device([pool.data_ptr() + i * slot for i in range(n)], [size] * n, None,
                    cuts.data_ptr(), counts.data_ptr(), _hs())
    torch.cuda.synchronize()
    c = cuts.cpu().numpy().view(np.uint64)
    k = counts.cpu().numpy()
    starts = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    ends = [c[b:b + m] for b, m in zip(starts, k)]
    assert int(k.sum()) == g['chunks']
    assert G.cutlist_digest(ends) == g['sha256']
    del pool
    torch.cuda.empty_cache()
