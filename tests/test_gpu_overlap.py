"""GPU parity of pipelined calls (RC_PIPELINED, include/replicat_chunker.h): the tile kernel on
a CU-masked stream of most CUs, the edge and chain kernels on the reserved CUs, so that one
call's chain runs beside the next call's tile kernel.  Every cut must equal the reference's
(golden fixtures) and the sequential path's; the caller's stream orders the inputs and
rc_chunk_wait the outputs -- the tests read results through the caller's stream only
(``.cpu()`` synchronises that stream, not the device), so a missing wait shows as wrong data."""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from gpu_util import chunk_device, device_streams  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd._lib import ChunkerError  # noqa: E402
from replicat_amd.chunker import (MAX_LENGTH, MIN_LENGTH, GpuChunker,  # noqa: E402
                                  fill_splitmix, fill_splitmix_streams, normalize_params)

SMALL = G.load('small_cases.json')
STREAMS = G.load('streams.json')
MIB = 1 << 20


@pytest.fixture(autouse=True)
def _own_stream():
    """Callers of pipelined calls use a non-blocking stream: the legacy NULL stream would
    synchronise with the chunker's CU-masked streams (correct, but serial)."""
    with torch.cuda.stream(torch.cuda.Stream()):
        yield
    torch.cuda.synchronize()


def _hs():
    return torch.cuda.current_stream().cuda_stream


def _ends(cuts, counts, caps):
    c = cuts.cpu().numpy().view(np.uint64)
    k = counts.cpu().numpy()
    assert (k >= 0).all()
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    return [c[b:b + m].tolist() for b, m in zip(base, k)]


def test_overlap_split():
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    assert ch.overlap(0) == 32
    assert ch.overlap(8) == 8
    assert ch.overlap(32) == 32
    with pytest.raises(ChunkerError):
        ch.overlap(torch.cuda.get_device_properties(0).multi_processor_count)


@pytest.fixture
def pipe_all(monkeypatch):
    """RC_PIPE_ALL=1: every pipelined request on the masked streams (small batches and
    small-window chunkers otherwise run in sequence on the caller's stream)."""
    monkeypatch.setenv('RC_PIPE_ALL', '1')


@pytest.mark.parametrize('reserve,force', [(8, True), (32, False), (64, True)])
def test_small_cases_pipelined(reserve, force, monkeypatch):
    """Every small case (mixed lengths and framings per stream), one pipelined call per
    parameter set.  force: on the masked streams (RC_PIPE_ALL=1), else the library's choice
    (these small batches: in sequence)."""
    if force:
        monkeypatch.setenv('RC_PIPE_ALL', '1')
    cases = [c for c in SMALL if c['max'] % 4 == 0 or len(c['pieces']) <= 1]
    by_params = {}
    for c in cases:
        by_params.setdefault((c['min'], c['max'], normalize_params(G.params_of(c))), []).append(c)
    for (mn, mx, key), group in by_params.items():
        ch = GpuChunker(mn, mx, key)
        ch.overlap(reserve)
        datas = [np.frombuffer(b''.join(G.case_pieces(c)), np.uint8) for c in group]
        sizes = [c['size'] for c in group]
        last = [c['size'] - c['pieces'][-1] if c['pieces'] else 0 for c in group]
        ts = device_streams(sizes, datas=datas)
        ends = chunk_device(ch, ts, sizes, last, pipelined=True)
        for c, e in zip(group, ends):
            assert [b - a for a, b in zip([0] + e[:-1], e)] == c['expected']


def test_golden_streams_pipelined(pipe_all):
    """streams.json (64 MiB streams, 16 MiB piece framing, zero / constant data) pipelined."""
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
        got = chunk_device(ch, ts, sizes, last, pipelined=True)
        for e, g in zip(es, got):
            assert g == e['ends'], (e['data'], e['size'])


@pytest.mark.parametrize('tile_streams', [1, 2])
def test_back_to_back_batches(pipe_all, tile_streams, monkeypatch):
    """Eight pipelined calls over different batches (workspaces alternate while chains run
    beside later tile kernels), each with its own outputs, then mixed with sequential calls;
    one wait, then every batch against its sequential result.  tile_streams=2
    (RC_TILE_STREAMS): consecutive tile kernels on two masked streams, free to overlap."""
    monkeypatch.setenv('RC_TILE_STREAMS', str(tile_streams))
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    ch.overlap(16)
    n, size = 32, 16 * MIB
    pools, outs = [], []
    for b in range(8):
        pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 1000 * b, 1, _hs())
        pools.append(pool)
    total, caps = ch.capacity([size] * n)
    for b, pool in enumerate(pools):
        cuts = torch.full((total,), -7, dtype=torch.int64, device='cuda')
        counts = torch.full((n,), -7, dtype=torch.int64, device='cuda')
        # batches 3 and 6 run sequentially on the caller's stream between pipelined ones, and
        # the last ends the sequence (RC_PIPELINE_END: its chain on every CU)
        ch.chunk_device(np.arange(n, dtype=np.uint64) * size + pool.data_ptr(), [size] * n, None,
                        cuts.data_ptr(), counts.data_ptr(), _hs(), pipelined=b not in (3, 6),
                        end=b == 7)
        outs.append((cuts, counts))
    ch.wait(_hs())
    got = [_ends(c, k, caps) for c, k in outs]
    seq = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    for b, pool in enumerate(pools):
        ts = [pool[i * size:(i + 1) * size] for i in range(n)]
        assert got[b] == chunk_device(seq, ts, [size] * n), b


def test_inputs_ordered_by_caller_stream(pipe_all):
    """The bytes are generated on the caller's stream right before the pipelined call, with no
    synchronisation: the tile kernel must wait for them (streams.json's 64 MiB splitmix
    stream, then the same buffer overwritten and chunked again)."""
    e = next(x for x in STREAMS if x['data'][0] == 'splitmix' and x['params'] is None
             and x['min'] == MIN_LENGTH and x['max'] == MAX_LENGTH)
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    L, P = e['size'], G.last_piece_start(e['size'], e['piece'])
    t = torch.empty(L + 16, dtype=torch.uint8, device='cuda')
    total, caps = ch.capacity([L])
    res = []
    for fill in ('zero', 'golden', 'zero', 'golden'):
        if fill == 'zero':
            t.zero_()
        else:
            fill_splitmix(t.data_ptr(), L, e['data'][1], e['data'][2], _hs())
        cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
        counts = torch.zeros(1, dtype=torch.int64, device='cuda')
        ch.chunk_device([t.data_ptr()], [L], [P], cuts.data_ptr(), counts.data_ptr(), _hs(),
                        pipelined=True)
        # the next fill overwrites t: the caller's stream must not run ahead of the tile
        # kernel that reads it
        ch.wait(_hs())
        res.append(_ends(cuts, counts, caps)[0])
    assert res[1] == e['ends'] and res[3] == e['ends']
    assert res[0] == res[2] and res[0] != e['ends']


def test_reference_harness_stream_pipelined(pipe_all):
    g = G.load('harness.json')
    L = g['length']
    dev = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for piece in synth.harness_buffers(g['number'], g['size'], g['seed']):
        dev[off:off + len(piece)].copy_(torch.frombuffer(piece, dtype=torch.uint8))
        off += len(piece)
    ch = GpuChunker(g['min'], g['max'], b'\xff' * 16)
    for reserve in (8, 16, 32):
        ch.overlap(reserve)
        ends = chunk_device(ch, [dev], [L], [g['last_piece']], pipelined=True)[0]
        assert len(ends) == g['chunks'], reserve
        assert G.cutlist_digest([ends]) == g['sha256'], reserve
    del dev
    torch.cuda.empty_cache()


@pytest.mark.parametrize('name,force', [('config2_ff', False), ('config3iii', False),
                                        ('config3iii', True)])
def test_full_size_pipelined(name, force, monkeypatch):
    """Config 2 (1024 x 64 MiB: pipelined by default) and 3 (iii) (65,536 x 1 MiB at 2,000 /
    80,000: in sequence by default, on the masked streams with RC_PIPE_ALL=1) as three
    pipelined calls into three output buffers: each equals the reference's digest."""
    if force:
        monkeypatch.setenv('RC_PIPE_ALL', '1')
    g = {x['name']: x for x in G.load('digests.json')}[name]
    n, size = g['streams'], g['size']
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, g['seed'], 0, 1, _hs())
    key = b'\xff' * 16 if g.get('params') is None else bytes.fromhex(g['params'])
    ch = GpuChunker(g['min'], g['max'], key)
    total, caps = ch.capacity([size] * n)
    ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
    outs = []
    for _ in range(3):
        cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
        counts = torch.zeros(n, dtype=torch.int64, device='cuda')
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), _hs(),
                        pipelined=True)
        outs.append((cuts, counts))
    ch.wait(_hs())
    for cuts, counts in outs:
        ends = _ends(cuts, counts, caps)
        assert sum(len(e) for e in ends) == g['chunks']
        assert G.cutlist_digest(ends) == g['sha256']
    del pool, outs
    torch.cuda.empty_cache()


def test_pipeline_end_orders_shared_outputs(pipe_all):
    """RC_PIPELINE_END calls (chain on every CU) between ordinary pipelined ones, all writing
    the SAME output arrays from two different batches: the chains must stay in call order
    across the two chain streams, so the arrays end with the last call's cuts."""
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    n, size = 16, 16 * MIB
    pools = []
    for b in range(2):
        pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 500 * b, 1, _hs())
        pools.append(pool)
    total, caps = ch.capacity([size] * n)
    exp = []
    seq = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    for pool in pools:
        exp.append(chunk_device(seq, [pool[i * size:(i + 1) * size] for i in range(n)], [size] * n))
    assert exp[0] != exp[1]
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    plan = [(0, False), (1, True), (0, False), (1, False), (0, True), (1, True), (0, False)]
    for k in range(1, len(plan) + 1):
        for b, end in plan[:k]:
            ch.chunk_device(np.arange(n, dtype=np.uint64) * size + pools[b].data_ptr(), [size] * n,
                            None, cuts.data_ptr(), counts.data_ptr(), _hs(), pipelined=True,
                            end=end)
        ch.wait(_hs())
        assert _ends(cuts, counts, caps) == exp[plan[k - 1][0]], plan[:k]


@pytest.mark.parametrize('end', [False, True])
def test_sequential_after_pipelined_shares_outputs(end):
    """a call in sequence right after pipelined ones on the same chunker, into the
    SAME cut and count arrays, must end with its own cuts -- the pipelined calls' chains may
    still run on the reserved CUs' stream (end: on the every-CU stream of RC_PIPELINE_END) when
    the later call's chain starts on the caller's stream."""
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    size, na, nb = 16 * MIB, 48, 24
    a = torch.empty(na * size + 64, dtype=torch.uint8, device='cuda')
    b = torch.empty(nb * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(a.data_ptr(), na, size, size, synth.DEFAULT_SEED, 700, 1, _hs())
    fill_splitmix_streams(b.data_ptr(), nb, size, size, synth.DEFAULT_SEED, 3000, 1, _hs())
    seq = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    exp_b = chunk_device(seq, [b[i * size:(i + 1) * size] for i in range(nb)], [size] * nb)
    total, caps = ch.capacity([size] * na)
    _, caps_b = ch.capacity([size] * nb)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(na, dtype=torch.int64, device='cuda')
    pa = np.arange(na, dtype=np.uint64) * size + a.data_ptr()
    pb = np.arange(nb, dtype=np.uint64) * size + b.data_ptr()
    for rnd in range(3):
        for k in range(2):
            ch.chunk_device(pa, [size] * na, None, cuts.data_ptr(), counts.data_ptr(), _hs(),
                            pipelined=True, end=end and k == 1)
        before = ch.pipelined_calls()
        assert before == 2 * (rnd + 1)  # the A calls were pipelined
        ch.chunk_device(pb, [size] * nb, None, cuts.data_ptr(), counts.data_ptr(), _hs())
        assert ch.pipelined_calls() == before  # the B call ran in sequence
        ch.wait(_hs())
        got = _ends(cuts[:int(caps_b.sum())], counts[:nb], caps_b)
        assert got == exp_b, rnd
    del a, b
    torch.cuda.empty_cache()


@pytest.mark.parametrize('tile_streams', [1, 2])
def test_mixed_calls_share_outputs(pipe_all, tile_streams, monkeypatch):
    """pipelined and sequential calls alternate into ONE cuts / counts buffer (two
    batches whose streams land in the same slots), with one and two tile streams
    (RC_TILE_STREAMS): after every prefix of the sequence the buffer holds the last call's
    cuts, as a sequential chunker gives them."""
    monkeypatch.setenv('RC_TILE_STREAMS', str(tile_streams))
    ch = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    n, size = 16, 16 * MIB
    pools = []
    for b in range(2):
        pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 800 + 300 * b, 1,
                              _hs())
        pools.append(pool)
    total, caps = ch.capacity([size] * n)
    seq = GpuChunker(MIN_LENGTH, MAX_LENGTH, b'\xff' * 16)
    exp = [chunk_device(seq, [p[i * size:(i + 1) * size] for i in range(n)], [size] * n)
           for p in pools]
    assert exp[0] != exp[1]
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    plan = [(0, 'p'), (1, 's'), (0, 'p'), (1, 'p'), (0, 's'), (1, 'p'), (0, 'e'), (1, 's'),
            (0, 'p')]
    for k in (1, 2, 3, 5, 7, 8, 9):
        for b, how in plan[:k]:
            ch.chunk_device(np.arange(n, dtype=np.uint64) * size + pools[b].data_ptr(), [size] * n,
                            None, cuts.data_ptr(), counts.data_ptr(), _hs(), pipelined=how != 's',
                            end=how == 'e')
        ch.wait(_hs())
        assert _ends(cuts, counts, caps) == exp[plan[k - 1][0]], plan[:k]
