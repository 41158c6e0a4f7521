"""The tile kernel's work schedule (kernels.hip TileUnits): static ranges, then units grabbed
from a counter.  Since round 5 every launch hands out all its tiles as 3-tile units, 64 per
workgroup grab, so the ordinary parity tests run that schedule; here the same oracle checks run
under the older schedules (fully static, per-wave grabs) and other unit and group sizes, with
RC_TILE_DYN_MIN=0 (every launch dynamic), so unit switches land everywhere: inside streams,
on stream boundaries, on tiles the fast path does not take, on tie tiles (zeros: every tile
ties), in segmented chains.  The knobs are read when a chunker is created (knobs.h), and every
check creates its chunkers after monkeypatch.setenv.  Workgroup grabs (RC_TILE_GROUP: units
dealt to a workgroup's waves through LDS, kernels.hip UnitGrab) are followed by
rc_chunker_check (no fail-safe stop).  Tile records come back from a poisoned buffer (rc_tile_records), so a unit that no wave
ran shows as a wrong record."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import test_gpu_parity as P  # noqa: E402
from gpu_util import chunk_device, device_streams, expected_cuts, open_prefix  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402

# (static per mille, unit tiles, units per workgroup grab): fully static (round 2), the round-3/4
# per-wave grabs, small per-wave units, and workgroup grabs of 16 to 256 units (the default since
# round 5 is 0:3:64, which every other GPU test runs; groups below 16 run as 16 since round 6 --
# the LDS ring's margin, kernels.hip UnitGrab)
SCHEDULES = [('1000', '12', '0'), ('100', '12', '0'), ('0', '2', '0'), ('900', '7', '0'),
             ('0', '2', '16'), ('100', '3', '32'), ('0', '2', '256'), ('500', '5', '16')]


@pytest.fixture(params=SCHEDULES, ids=['s%s_c%s_g%s' % x for x in SCHEDULES])
def dynamic(request, monkeypatch):
    st, ck, grp = request.param
    monkeypatch.setenv('RC_TILE_DYN_MIN', '0')
    monkeypatch.setenv('RC_TILE_STATIC', st)
    monkeypatch.setenv('RC_TILE_CHUNK', ck)
    monkeypatch.setenv('RC_TILE_GROUP', grp)
    return request.param


@pytest.mark.parametrize('seed', [0, 2, 5])
def test_random_vs_oracle_dynamic(dynamic, seed):
    P.test_random_vs_oracle(seed)


@pytest.mark.parametrize('kind', ['random', 'zeros', 'periodic', 'framed'])
def test_tile_records_dynamic(dynamic, kind):
    P.test_tile_records_vs_oracle(kind)


@pytest.mark.parametrize('kind', ['random', 'zeros'])
def test_tile_group_maxima_dynamic(dynamic, kind):
    P.test_tile_group_maxima_vs_oracle(kind)


def test_segmented_chains_dynamic(dynamic, monkeypatch):
    P.test_segmented_chains_vs_oracle(monkeypatch, 1 << 16, 1, '0')


def test_many_small_streams_dynamic(dynamic):
    """Units spanning many streams (the cursor re-seeks at every unit switch)."""
    o = P._oracle()
    mn, mx = 64, 4096
    key = synth.seeded_key(21)
    ch = GpuChunker(mn, mx, key)
    rnd = np.random.default_rng(5)
    sizes = [int(x) for x in rnd.integers(0, 70_000, 600)]
    datas = [synth.stream_bytes(n, synth.DEFAULT_SEED, 900 + i) for i, n in enumerate(sizes)]
    last = [int(rnd.integers(0, n + 1)) if n else 0 for n in sizes]
    ts = device_streams(sizes, datas=datas)
    got = chunk_device(ch, ts, sizes, last)
    for g, e in zip(got, expected_cuts(datas, mn, mx, key, last)):
        assert g == e


@pytest.mark.parametrize('sched', ['1000:12:128:0', '100:2:0:0', '100:2:0:32'])
def test_harness_stream_schedules(monkeypatch, sched):
    """The reference harness's stream (one 5.12 GB stream, ~76 tiles per wave: fully static by
    default until round 5, workgroup grabs of 3-tile units since) under the round-4 static
    schedule, per-wave grabs and workgroup grabs of 2-tile units: the cut list equals the
    reference's (tests/golden/harness.json)."""
    st, ck, dm, grp = sched.split(':')
    monkeypatch.setenv('RC_TILE_DYN_MIN', dm)
    monkeypatch.setenv('RC_TILE_STATIC', st)
    monkeypatch.setenv('RC_TILE_CHUNK', ck)
    monkeypatch.setenv('RC_TILE_GROUP', grp)
    import golden_util as G
    pieces = list(synth.harness_buffers())
    L = sum(len(p) for p in pieces)
    pool = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for p in pieces:
        pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
        off += len(p)
    ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
    total, caps = ch.capacity([L])
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(1, dtype=torch.int64, device='cuda')
    for _ in range(2):  # the second call reuses the first's records buffer
        cuts.zero_()
        ch.chunk_device([pool.data_ptr()], [L], [L - len(pieces[-1])], cuts.data_ptr(),
                        counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ch.check()
        k = int(counts.cpu()[0])
        ends = cuts[:k].cpu().numpy().view(np.uint64)
        assert G.cutlist_digest([ends]) == G.load('harness.json')['sha256']
    del pool
    torch.cuda.empty_cache()


def test_constant_data_default_schedule():
    """8 GiB of zeros in one launch under the DEFAULT schedule (grabbed units): every tile is a
    tie tile, resolved by the edge kernel from the per-unit lists; 16 identical streams, each
    checked against the oracle's cut list of one of them."""
    o = P._oracle()
    n, size = 16, 512 << 20
    ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
    pool = torch.zeros(n * size + 64, dtype=torch.uint8, device='cuda')
    exp = o.chunk_stream(np.zeros(size, np.uint8), 128_000, 5_120_000, None, 0)
    total, caps = ch.capacity([size] * n)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    ch.chunk_device([pool.data_ptr() + i * size for i in range(n)], [size] * n, None,
                    cuts.data_ptr(), counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = cuts.cpu().numpy().view(np.uint64)
    k = counts.cpu().numpy()
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    for i in range(n):
        assert c[base[i]:base[i] + k[i]].tolist() == exp, i
    del pool
    torch.cuda.empty_cache()


def test_fresh_chunkers_first_call_on_a_nonblocking_stream():
    """Round 5: every launch grabs its units from the workspace's counter, and a NEW workspace's
    counter was zeroed by hipMemset on the NULL stream, which a non-blocking caller stream does
    not wait for -- a fresh chunker's first call once came back with garbage counts.  Fresh
    chunkers, each called once from a non-blocking stream right after creation (small launches,
    where the first tile kernel starts soonest), must all match the oracle."""
    o = P._oracle()
    mn, mx = 2_000, 80_000
    sizes = [1 << 20, 3 << 20, 777_777, 5 << 20]
    datas = [synth.stream_bytes(n, synth.DEFAULT_SEED, 60 + i) for i, n in enumerate(sizes)]
    exp = expected_cuts(datas, mn, mx, None, [0] * len(sizes))
    with torch.cuda.stream(torch.cuda.Stream()):
        ts = device_streams(sizes, datas=datas)
        for _ in range(24):
            ch = GpuChunker(mn, mx, b'\xff' * 16)
            assert chunk_device(ch, ts, sizes, [0] * len(sizes)) == exp
            ch.check()
            ch.close()
    torch.cuda.synchronize()
    assert o is not None
