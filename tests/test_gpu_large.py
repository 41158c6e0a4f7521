"""GPU parity at the large configurations of SURVEY.md §8(d) against the reference's golden
values (tests/golden/large.json, made by make_golden.py --large from the reference adapter):

* config 3 (ii): one 64 GiB stream, last piece the final 1 MiB -- as one device stream and as
  the multi-device split (replicat_amd/split.py) simulated window by window on one GPU;
* config 5: the re-chunk of config 2 with 512 edited copies and its dedup ratio.
"""
import types

import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import bench  # noqa: E402
from gpu_util import chunk_device, device_streams  # noqa: E402

from replicat_amd import split, synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix, fill_splitmix_at  # noqa: E402

LARGE = {d['name']: d for d in G.load('large.json')}


def _hs():
    return torch.cuda.current_stream().cuda_stream


def test_fill_at_offset_matches_host():
    t = torch.empty(4096 + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_at(t.data_ptr(), 4093, synth.DEFAULT_SEED, 3, 1000, _hs())
    got = t[:4093].cpu().numpy()
    exp = synth.stream_bytes(8000 + 4093, synth.DEFAULT_SEED, 3)[8000:]
    assert np.array_equal(got, exp)


def _window_runner(ch, windows_bufs):
    """chunk_window over per-window device buffers (one GPU standing in for the ranks)."""
    fake = types.SimpleNamespace(ch=ch, hs=_hs())

    def run(w, entry):
        buf = windows_bufs[w.start]
        st = bench.Config3ii.__new__(bench.Config3ii)
        st.ch, st.hs, st.buf = ch, fake.hs, buf
        st.be = bench.Backend(torch.cuda.current_device())
        _, caps = ch.capacity([w.end - w.start])
        st.cap = int(caps[0])
        st.cuts = torch.zeros(st.cap + 1, dtype=torch.int64, device='cuda')
        st.counts = torch.zeros(1, dtype=torch.int64, device='cuda')
        return bench.Config3ii.chunk_window(st, w, entry)
    return run


@pytest.mark.parametrize('world', [2, 3, 8])
def test_split_small_vs_oracle(world, oracle):
    mn, mx = 2_000, 80_000
    key = synth.seeded_key(4)
    L = 40_000_000 + 12
    P = L - (1 << 20)
    data = synth.stream_bytes(L, synth.DEFAULT_SEED, 11)
    exp = oracle.chunk_stream(data, mn, mx, key, P)
    ch = GpuChunker(mn, mx, key)
    windows = split.plan_windows(L, P, world, mx)
    bufs = {}
    for w in windows:
        t = torch.empty(w.end - w.start + 64, dtype=torch.uint8, device='cuda')
        t[:w.end - w.start].copy_(torch.from_numpy(np.ascontiguousarray(data[w.start:w.end])))
        bufs[w.start] = t
    run = _window_runner(ch, bufs)
    chains = [(w.start, run(w, w.start)) for w in windows]
    # force one exact fallback too: window 1's speculative list shifted off the grid
    variants = [chains, [chains[0], (chains[1][0], [e + 2 for e in chains[1][1]])] + chains[2:]]
    for cs in variants:
        cs = list(cs)
        while True:
            ends, r, entry = split.splice(windows, cs)
            if r is None:
                break
            cs[r] = (entry, run(windows[r], entry))
        assert ends == exp


def test_config3ii_single_stream():
    d = LARGE['config3ii']
    ch = GpuChunker(d['min'], d['max'], b'\xff' * 16)
    ts = device_streams([d['size']], seed=d['seed'], ids=[d['stream']])
    ends = chunk_device(ch, ts, [d['size']], [d['last_piece']])[0]
    assert ends[:64] == d['first_ends'] and ends[-16:] == d['last_ends']
    assert len(ends) == d['chunks'] and G.cutlist_digest([ends]) == d['sha256']
    del ts
    torch.cuda.empty_cache()


@pytest.mark.parametrize('world', [4])
def test_config3ii_split_windows(world):
    """The multi-GPU split of config 3 (ii), its windows chunked one after another here."""
    d = LARGE['config3ii']
    ch = GpuChunker(d['min'], d['max'], b'\xff' * 16)
    windows = split.plan_windows(d['size'], d['last_piece'], world, d['max'])
    chains = []
    for w in windows:
        t = torch.empty(w.end - w.start + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_at(t.data_ptr(), w.end - w.start, d['seed'], d['stream'], w.start // 8,
                         _hs())
        run = _window_runner(ch, {w.start: t})
        chains.append((w.start, run(w, w.start)))
        del t, run
        torch.cuda.empty_cache()
    ends, r, _ = split.splice(windows, chains)
    assert r is None  # the chains meet inside the halo
    assert len(ends) == d['chunks'] and G.cutlist_digest([ends]) == d['sha256']


def test_config5_dedup():
    d = LARGE['config5']
    ch = GpuChunker(d['min'], d['max'], b'\xff' * 16)
    n, size = d['streams'], d['size']
    slot = size + 64
    pool = torch.empty(n * slot + 64, dtype=torch.uint8, device='cuda')
    for i in range(n):
        fill_splitmix(pool.data_ptr() + i * slot, size, d['seed'], i, _hs())
    c5 = bench.Config5(ch, pool, slot, n, size, 0, _hs())
    assert c5.orig_digest == d['original_sha256']
    total, caps = ch.capacity(c5.lens)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    ch.chunk_device(c5.ptrs, c5.lens, None, cuts.data_ptr(), counts.data_ptr(), _hs())
    _, _, ends = bench.cut_digest(cuts, counts, caps)
    assert G.cutlist_digest([ends[i] for i in c5.edited]) == d['edited_sha256']
    assert [e.tolist() for e in (ends[i] for i in c5.edited[:6])] == d['edited_first_ends']
    r = c5.dedup(ends)
    assert r['dup_bytes_edited'] == d['dup_bytes_edited']
    assert r['total_bytes_edited'] == d['total_bytes_edited']
    del pool, c5
    torch.cuda.empty_cache()
