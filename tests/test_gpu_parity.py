"""GPU parity: the HIP chunker (through the C ABI) against the reference's golden outputs and
the oracle, bit for bit.  Runs on an MI355X only (-m gpu)."""
import random

import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from gpu_util import chunk_device, device_streams, expected_cuts, open_prefix  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd._replicat_adapters import _gclmulchunker  # noqa: E402
from replicat_amd.adapters import gclmulchunker as BatchedChunker  # noqa: E402
from replicat_amd.chunker import GpuChunker, normalize_params  # noqa: E402

SMALL = G.load('small_cases.json')
KNOWN = G.load('known_answers.json')
STREAMS = G.load('streams.json')
DIGESTS = G.load('digests.json')


def loop_next_cut(pieces, min_length, max_length, params):
    """replicat's adapter loop (replicat/utils/adapters.py:290-305) over the drop-in
    `_gclmulchunker`: the reference's caller, unchanged, on top of the HIP module."""
    chunker = _gclmulchunker(min_length, max_length, normalize_params(params))
    buffer = bytearray()
    sizes = []
    it = iter(pieces)
    chunk = next(it, None)
    while chunk is not None:
        buffer += chunk
        nxt = next(it, None)
        while True:
            pos = chunker.next_cut(buffer, bool(nxt is None))
            if not pos:
                break
            sizes.append(pos)
            del buffer[:pos]
        chunk = nxt
    return sizes


def batched(pieces, min_length, max_length, params, batch_bytes):
    c = BatchedChunker(min_length=min_length, max_length=max_length, batch_bytes=batch_bytes)
    out = list(c(pieces, params=params))
    assert b''.join(out) == b''.join(pieces)
    return [len(x) for x in out]


@pytest.mark.parametrize('idx', range(0, len(SMALL), 3))
def test_small_cases_next_cut_loop(idx):
    case = SMALL[idx]
    if case['max'] % 4 and len(case['pieces']) > 1:
        pytest.skip('outside the parity domain (SURVEY.md §8 a0 S7)')
    got = loop_next_cut(G.case_pieces(case), case['min'], case['max'], G.params_of(case))
    assert got == case['expected']


def test_small_cases_device_batch():
    """All small cases in ONE rc_chunk_device call (mixed lengths / framings per stream)."""
    cases = [c for c in SMALL if c['max'] % 4 == 0 or len(c['pieces']) <= 1]
    by_params = {}
    for c in cases:
        by_params.setdefault((c['min'], c['max'], normalize_params(G.params_of(c))), []).append(c)
    for (mn, mx, key), group in by_params.items():
        ch = GpuChunker(mn, mx, key)
        datas = [np.frombuffer(b''.join(G.case_pieces(c)), np.uint8) for c in group]
        sizes = [c['size'] for c in group]
        last = [c['size'] - c['pieces'][-1] if c['pieces'] else 0 for c in group]
        ts = device_streams(sizes, datas=datas)
        ends = chunk_device(ch, ts, sizes, last)
        for c, e in zip(group, ends):
            assert [b - a for a, b in zip([0] + e[:-1], e)] == c['expected']


@pytest.mark.parametrize('batch_bytes', [1 << 12, 1 << 16, 1 << 28])
def test_small_cases_batched_adapter(batch_bytes):
    for case in SMALL[::2]:
        if case['max'] % 4:
            continue
        got = batched(G.case_pieces(case), case['min'], case['max'], G.params_of(case),
                      batch_bytes)
        assert got == case['expected'], case


@pytest.mark.parametrize('idx', range(len(KNOWN['alignment'])))
def test_known_alignment(idx):
    c = KNOWN['alignment'][idx]
    pieces = [bytes([c['byte']]) * n for n in c['pieces']]
    assert loop_next_cut(pieces, c['min'], c['max'], None) == c['expected']
    if c['max'] % 4 == 0:
        assert batched(pieces, c['min'], c['max'], None, 1) == c['expected']


@pytest.mark.parametrize('idx', range(len(KNOWN['seeded'])))
def test_known_seeded(idx):
    c = KNOWN['seeded'][idx]
    pieces = G.seeded_inputs(c)
    params = bytes.fromhex(c['params'])
    assert batched(pieces, 500, 10_000, params, 1 << 20) == c['expected']
    if c['repeat'] == 1:
        assert loop_next_cut(pieces, 500, 10_000, params) == c['expected']
    if 'expected_after_flip0' in c:
        data = bytearray(pieces[0])
        data[0] = (data[0] - 1) % 255
        assert batched([bytes(data)], 500, 10_000, params, 1 << 20) == c['expected_after_flip0']


def test_golden_streams_device():
    """streams.json: 64 MiB streams, 16 MiB piece framing, zero / constant data, 1 MiB."""
    groups = {}
    for e in STREAMS:
        key = normalize_params(None if e['params'] is None else bytes.fromhex(e['params']))
        groups.setdefault((e['min'], e['max'], key), []).append(e)
    for (mn, mx, key), es in groups.items():
        ch = GpuChunker(mn, mx, key)
        ts, sizes, last = [], [], []
        for e in es:
            sizes.append(e['size'])
            last.append(G.last_piece_start(e['size'], e['piece']))
            if e['data'][0] == 'splitmix':
                ts += device_streams([e['size']], seed=e['data'][1], ids=[e['data'][2]])
            else:
                ts += device_streams([e['size']], fill=e['data'][1])
        got = chunk_device(ch, ts, sizes, last)
        for e, g in zip(es, got):
            assert g == e['ends'], (e['data'], e['size'])


@pytest.mark.parametrize('name', [d['name'] for d in DIGESTS])
def test_full_size_digests(name):
    """Full configuration sizes, device-generated bytes: SHA-256 of all cut lists equals the
    reference's (config 2 = 1024 x 64 MiB, 64 GiB resident in HBM)."""
    d = next(x for x in DIGESTS if x['name'] == name)
    key = normalize_params(None if d['params'] is None else bytes.fromhex(d['params']))
    ch = GpuChunker(d['min'], d['max'], key)
    all_ends = []
    per_call = max(1, (16 << 30) // d['size'])
    for first in range(0, d['streams'], per_call):
        ids = list(range(first, min(d['streams'], first + per_call)))
        ts = device_streams([d['size']] * len(ids), seed=d['seed'], ids=ids)
        all_ends += chunk_device(ch, ts, [d['size']] * len(ids))
        del ts
        torch.cuda.empty_cache()
    assert sum(map(len, all_ends)) == d['chunks']
    assert G.cutlist_digest(all_ends) == d['sha256']


def _oracle():
    from oracle import oracle as o
    o.lib()
    return o


@pytest.mark.parametrize('seed', range(6))
def test_random_vs_oracle(seed):
    """Random params/framing/data (incl. long runs of equal keys) against the oracle."""
    o = _oracle()
    rnd = random.Random(seed)
    mx = rnd.choice([8, 64, 4096, 16384 + 4, 65536, 1 << 20])
    mn = rnd.randrange(1, mx + 1)
    key = rnd.randbytes(16)
    if key[:8] == bytes(8):
        key = b'\x01' + key[1:]
    ch = GpuChunker(mn, mx, key)
    sizes, datas, last = [], [], []
    for _ in range(24):
        n = rnd.choice([0, 3, 8, mx, 2 * mx, 2 * mx + 5, rnd.randrange(0, 40 * mx + 1),
                        rnd.randrange(0, 8 << 20)])
        kind = rnd.random()
        if kind < 0.7:
            d = np.frombuffer(rnd.randbytes(n), np.uint8)
        elif kind < 0.8:
            d = np.zeros(n, np.uint8)
        else:
            unit = np.frombuffer(rnd.randbytes(rnd.randrange(1, 64)), np.uint8)
            d = np.resize(unit, n)
        sizes.append(n)
        datas.append(d)
        last.append(rnd.choice([0, n, rnd.randrange(0, n + 1)]))
    ts = device_streams(sizes, datas=datas)
    got = chunk_device(ch, ts, sizes, last)
    for d, P, g, e in zip(datas, last, got, expected_cuts(datas, mn, mx, key, last)):
        assert g == e, (mn, mx, len(d), P)


def test_open_prefix_matches_nonfinal_calls():
    """RC_OPEN: cuts only while L - s >= max (the adapter's non-final next_cut calls)."""
    o = _oracle()
    mn, mx = 500, 10_000
    key = b'\x5a' * 16
    ch = GpuChunker(mn, mx, key)
    rnd = random.Random(7)
    data = np.frombuffer(rnd.randbytes(3_000_000), np.uint8)
    ts = device_streams([data.size], datas=[data])
    got = chunk_device(ch, ts, [data.size], None, open_=True)[0]
    full = o.chunk_stream(data, mn, mx, key, data.size)  # P = L: argmax iff L - s >= max
    exp = []
    s = 0
    for e in full:
        if data.size - s < mx:
            break
        exp.append(e)
        s = e
    assert got == exp


def test_misaligned_and_bad_framing_rejected():
    ch = GpuChunker(500, 10_000, b'\xff' * 16)
    t = torch.zeros(1024, dtype=torch.uint8, device='cuda')
    from replicat_amd._lib import ChunkerError
    with pytest.raises(ChunkerError):
        ch.chunk_device([t.data_ptr() + 4], [100], [0], t.data_ptr(), t.data_ptr(), 0)
    with pytest.raises(ChunkerError):
        ch.chunk_device([t.data_ptr()], [100], [101], t.data_ptr(), t.data_ptr(), 0)


def test_host_path_matches_device():
    ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
    bufs = [synth.stream_bytes(n, synth.DEFAULT_SEED, i)
            for i, n in enumerate([64 << 20, 0, 5, 11 << 20, 48 << 20])]
    o = _oracle()
    got = ch.chunk_host(bufs)
    for b, g in zip(bufs, got):
        assert g.tolist() == o.chunk_stream(b, 128_000, 5_120_000, None, 0)


@pytest.mark.parametrize('kind', ['random', 'zeros', 'periodic', 'seeded_key', 'framed'])
def test_tile_records_vs_oracle(kind):
    """Phase A alone: every tile record (first maximal exact key, index) equals the oracle's.
    'framed': last pieces near the stream end put jneed within a tile of the last key, so the
    last tile runs past the data and takes the edge kernel (the others take the fast path)."""
    import ctypes
    o = _oracle()
    from replicat_amd.chunker import keys_needed, tile_keys
    tk = tile_keys()
    key = synth.seeded_key(9) if kind == 'seeded_key' else b'\xff' * 16
    mn, mx = 128_000, 5_120_000
    ch = GpuChunker(mn, mx, key)
    sizes = [(16 << 20) + 4 * 777, 12 << 20, 5 << 20]
    rnd = np.random.default_rng(3)
    if kind == 'zeros':
        datas = [np.zeros(n, np.uint8) for n in sizes]
    elif kind == 'periodic':
        datas = [np.resize(rnd.integers(0, 256, 4096 + 12, dtype=np.uint8), n) for n in sizes]
    else:
        datas = [synth.stream_bytes(n, synth.DEFAULT_SEED, 100 + i) for i, n in enumerate(sizes)]
    last = [0] * len(sizes)
    if kind == 'framed':
        last = [n - d for n, d in zip(sizes, (100, 4 * 4096 + 8, 1))]
    ts = device_streams(sizes, datas=datas)
    keys, js = ch.tile_records([t.data_ptr() for t in ts], sizes, last)
    k0 = int.from_bytes(key[:8], 'little')
    k1 = int.from_bytes(key[8:], 'little')
    base = 0
    for d, n, P in zip(datas, sizes, last):
        jneed = keys_needed(mx, n, P)
        nt = jneed // tk + 1 if jneed else 0
        ek = np.zeros(max(nt, 1), np.uint64)
        ej = np.zeros(max(nt, 1), np.uint64)
        buf = np.concatenate([d, np.zeros(16, np.uint8)])
        o.lib().oc_tile_records(k0, k1, buf.ctypes.data, n, jneed, tk, nt, ek.ctypes.data,
                                ej.ctypes.data)
        gk, gj = keys[base:base + nt], js[base:base + nt]
        bad = np.nonzero((gk != ek[:nt]) | ((gj != ej[:nt]) & (ek[:nt] != 0)))[0]
        assert bad.size == 0, (kind, n, bad[:8].tolist(), gk[bad[:4]].tolist(), ek[bad[:4]].tolist(),
                               gj[bad[:4]].tolist(), ej[bad[:4]].tolist())
        base += nt


@pytest.mark.parametrize('kind', ['random', 'zeros', 'periodic', 'seeded_key'])
def test_tile_group_maxima_vs_oracle(kind):
    """Small-window chunkers: the tile kernel's per-quarter group bounds (top-16 maxima and the
    lanes holding a key at or above the hot threshold) equal the oracle's for every fast tile;
    a tile sent to the exact path (the stream ends inside it, or a tie) reports ~0 and every
    lane hot, the no-bound values."""
    o = _oracle()
    from replicat_amd.chunker import keys_needed, tile_keys
    tk = tile_keys()
    key = synth.seeded_key(11) if kind == 'seeded_key' else b'\xff' * 16
    mn, mx = 2_000, 80_000
    ch = GpuChunker(mn, mx, key)
    sizes = [(3 << 20) + 4 * 321, 1 << 20, 200_004, 1000]
    rnd = np.random.default_rng(7)
    if kind == 'zeros':
        datas = [np.zeros(n, np.uint8) for n in sizes]
    elif kind == 'periodic':
        datas = [np.resize(rnd.integers(0, 256, 777, dtype=np.uint8), n) for n in sizes]
    else:
        datas = [synth.stream_bytes(n, synth.DEFAULT_SEED, 300 + i) for i, n in enumerate(sizes)]
    last = [0, (1 << 20) - 100, 0, 0]
    ts = device_streams(sizes, datas=datas)
    keys, js, gm, gh, hot = ch.tile_records([t.data_ptr() for t in ts], sizes, last, groups=True)
    assert 60000 < hot < 65536  # max 80,000: a window of 19,999 keys
    k0 = int.from_bytes(key[:8], 'little')
    k1 = int.from_bytes(key[8:], 'little')
    base = exact = 0
    none = np.uint64(2**64 - 1)
    for d, n, P in zip(datas, sizes, last):
        jneed = keys_needed(mx, n, P)
        nt = jneed // tk + 1 if jneed else 0
        eg = np.zeros(max(nt, 1), np.uint64)
        eh = np.zeros((max(nt, 1), 4), np.uint64)
        buf = np.concatenate([d, np.zeros(16, np.uint8)])
        # a stream's last tile is read up to the slice holding jneed (round 6, oc_clip_end)
        o.lib().oc_tile_groups(k0, k1, buf.ctypes.data, n, jneed, tk, nt, 4, eg.ctypes.data)
        o.lib().oc_tile_groups_hot(k0, k1, buf.ctypes.data, n, jneed, tk, nt, 4, hot,
                                   eh.ctypes.data)
        g, h = gm[base:base + nt], gh[base:base + nt]
        computed = g != none  # a tile sent to the exact path has no bounds at all
        ok = (((g == eg[:nt]) & (h == eh[:nt]).all(axis=1)) |
              (~computed & (h == none).all(axis=1)))
        assert ok.all(), (kind, n, np.nonzero(~ok)[0][:8].tolist())
        exact += int((~computed & (eg[:nt] != none)).sum())
        base += nt
    if kind in ('random', 'seeded_key'):
        assert exact <= 2  # ties inside a lane are rare on random data


@pytest.mark.parametrize('mode', ['repair', 'norepair', 'walk'])
@pytest.mark.parametrize('seg_bytes,ext', [(1 << 16, 0), (1 << 16, 1), (1 << 16, 4),
                                           (12 * 4096, 2), (1 << 20, 3), (1 << 12, 3)])
def test_segmented_chains_vs_oracle(monkeypatch, seg_bytes, ext, mode):
    """Segment-parallel speculative chains + join, with tiny segments and short extensions
    (ext 0: most boundaries miss).  repair: the merge kernel runs a missing boundary's chain on
    until the lists meet (the default); norepair (RC_REPAIR=0): any miss sends the stream to the
    sequential join; walk (RC_JOIN_WALK=1): every stream through the sequential join.  4 KiB
    segments are shorter than most chunks: extensions run past the next boundary's merge and
    the scan's entry recurrence skips lists (tests/test_join_model.py restates the splice)."""
    o = _oracle()
    monkeypatch.setenv('RC_JOIN_WALK', '1' if mode == 'walk' else '0')
    monkeypatch.setenv('RC_REPAIR', '0' if mode == 'norepair' else '1')
    monkeypatch.setenv('RC_SEGMENT_BYTES', str(seg_bytes))
    monkeypatch.setenv('RC_SEGMENT_EXT', str(ext))
    rnd = random.Random(seg_bytes + ext)
    for trial in range(3):
        mx = rnd.choice([4096, 16384, 4096 * 3])
        mn = rnd.choice([4, 500, mx // 2, mx])
        key = rnd.randbytes(16) if trial else b'\xff' * 16
        if key[:8] == bytes(8):
            key = b'\x01' + key[1:]
        ch = GpuChunker(mn, mx, key)
        sizes, datas, last = [], [], []
        for k in range(12):
            n = rnd.choice([rnd.randrange(0, 3 << 20), 2 << 20, (1 << 20) + 3, 7 * mx])
            kind = k % 4
            if kind == 0:
                d = np.frombuffer(rnd.randbytes(n), np.uint8)
            elif kind == 1:
                d = np.zeros(n, np.uint8)
            elif kind == 2:
                d = np.resize(np.frombuffer(rnd.randbytes(rnd.randrange(1, 9000)), np.uint8), n)
            else:
                d = synth.stream_bytes(n, synth.DEFAULT_SEED, 500 + k)
            sizes.append(n)
            datas.append(d)
            last.append(rnd.choice([0, n, rnd.randrange(0, n + 1)]))
        ts = device_streams(sizes, datas=datas)
        got = chunk_device(ch, ts, sizes, last)
        for d, P, g, e in zip(datas, last, got, expected_cuts(datas, mn, mx, key, last)):
            assert g == e, (mn, mx, len(d), P)
        got_open = chunk_device(ch, ts, sizes, None, open_=True)
        for d, g, full in zip(datas, got_open, expected_cuts(datas, mn, mx, key, sizes)):
            assert g == open_prefix(full, len(d), mx)
