"""GPU parity of the per-stream chains for small windows and many single-segment streams
(kernels.hip rc_quad_chain_kernel: a quad of lanes per stream; rc_lane_chain_kernel: one lane),
each walking its stream's cut chain from the tile records and the group bounds.  Every cut list
against the oracle (the reference's next_cut restated, oracle/gclmul_oracle.c), with the quad
chain forced (RC_LANE_CHAIN=1), the lane chain (=lane) and, for comparison, neither (=0: the
wave-per-stream spec kernel).  Runs on an MI355X only (-m gpu)."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from gpu_util import chunk_device, device_streams, expected_cuts, open_prefix  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402


def _oracle():
    from oracle import oracle as o
    o.lib()
    return o


def _data(rnd, kind, n, k):
    if kind == 'random':
        return np.frombuffer(rnd.randbytes(n), np.uint8)
    if kind == 'zeros':
        return np.zeros(n, np.uint8)
    if kind == 'periodic':  # long runs of equal keys: ties in every group
        return np.resize(np.frombuffer(rnd.randbytes(rnd.randrange(1, 6000)), np.uint8), n)
    if kind == 'sparse':  # mostly zero with a few random bytes: keys repeat inside lanes
        d = np.zeros(n, np.uint8)
        if n:
            idx = np.frombuffer(rnd.randbytes(8 * max(1, n // 4096)), np.uint64) % np.uint64(n)
            d[idx.astype(np.int64)] = 0xA5
        return d
    return synth.stream_bytes(n, synth.DEFAULT_SEED, 900 + k)


# (min, max): the config 3 (iii) pair, tiny windows inside one or two tiles, a window of 7.99
# tiles (the lane chain's widest: 8 full-tile records in flight), min = max, a min of one key step
PARAMS = [(2000, 80000), (500, 16384), (80000, 80000), (4, 4096 * 3), (12000, 131072),
          (64, 4096), (8, 3000)]


@pytest.mark.parametrize('lane', ['1', 'lane', '0'])
@pytest.mark.parametrize('mn,mx', PARAMS)
@pytest.mark.parametrize('kind', ['random', 'zeros', 'periodic', 'sparse', 'splitmix'])
def test_lane_chain_vs_oracle(monkeypatch, lane, mn, mx, kind):
    o = _oracle()
    monkeypatch.setenv('RC_LANE_CHAIN', lane)
    rnd = random.Random(f'{mn}-{mx}-{kind}')
    key = b'\xff' * 16 if kind != 'splitmix' else synth.seeded_key(5)
    ch = GpuChunker(mn, mx, key)
    sizes, datas, last = [], [], []
    for k in range(160):
        n = rnd.choice([0, 1, 7, 8, 4096, 16383, mx - 1, mx, mx + 3, 2 * mx - 4, 2 * mx + 5,
                        3 * mx + 1, rnd.randrange(0, 600_000), 1 << 20])
        n = max(n, 0)
        sizes.append(n)
        datas.append(_data(rnd, kind, n, k))
        last.append(rnd.choice([0, 0, n, rnd.randrange(0, n + 1)]))
    ts = device_streams(sizes, datas=datas)
    got = chunk_device(ch, ts, sizes, last)
    for d, P, g, e in zip(datas, last, got, expected_cuts(datas, mn, mx, key, last)):
        assert g == e, (mn, mx, kind, len(d), P)
    # non-final prefixes (RC_OPEN): argmax cuts only, no tail rule
    got_open = chunk_device(ch, ts, sizes, None, open_=True)
    fulls = expected_cuts(datas, mn, mx, key, sizes)
    for d, g, full in zip(datas, got_open, fulls):
        assert g == open_prefix(full, len(d), mx), (mn, mx, kind, len(d))


def test_lane_chain_many_streams_default_switch(monkeypatch):
    """No knob: a batch of >= 256 single-segment streams with the config 3 (iii) parameters
    takes the lane chain; a sample of its streams against the oracle, and every stream against
    the wave-per-stream chain."""
    o = _oracle()
    monkeypatch.delenv('RC_LANE_CHAIN', raising=False)
    mn, mx = 2000, 80000
    ch = GpuChunker(mn, mx, b'\xff' * 16)
    n, size = 2048, 256 << 10
    ts = device_streams([size] * n, seed=synth.DEFAULT_SEED, ids=list(range(4000, 4000 + n)))
    got = chunk_device(ch, ts, [size] * n)
    monkeypatch.setenv('RC_LANE_CHAIN', '0')  # read when a chunker is created (knobs.h)
    ref = chunk_device(GpuChunker(mn, mx, b'\xff' * 16), ts, [size] * n)
    assert got == ref
    for i in range(0, n, 97):
        d = ts[i][:size].cpu().numpy()
        assert got[i] == o.chunk_stream(d, mn, mx, b'\xff' * 16, 0), i
