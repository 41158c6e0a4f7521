"""Host side of GpuChunker.chunk_device (no GPU): the flags it hands the C ABI for each
combination of open_ / pipelined / end, and the stream arrays it builds."""
import numpy as np
import pytest

from replicat_amd import chunker as C
from replicat_amd._lib import RC_OPEN, RC_PIPELINE_END, RC_PIPELINED


class FakeLib:
    def __init__(self):
        self.calls = []

    def rc_chunk_device(self, h, n, ptrs, lens, last, flags, cuts, counts, stream):
        self.calls.append((n, flags, cuts, counts, stream))
        return 0


@pytest.fixture
def fake(monkeypatch):
    f = FakeLib()
    monkeypatch.setattr(C, 'lib', lambda: f)
    ch = object.__new__(C.GpuChunker)
    ch._h = 1
    yield ch, f
    ch._h = None


@pytest.mark.parametrize('open_,pipelined,end,flags', [
    (False, False, False, 0),
    (True, False, False, RC_OPEN),
    (False, True, False, RC_PIPELINED),
    (False, True, True, RC_PIPELINED | RC_PIPELINE_END),
    (True, True, True, RC_OPEN | RC_PIPELINED | RC_PIPELINE_END),
    (False, False, True, 0),  # end only means something for a pipelined call
])
def test_flags(fake, open_, pipelined, end, flags):
    ch, f = fake
    ch.chunk_device([16, 32], [100, 200], [0, 50], 1234, 5678, 9, open_, pipelined=pipelined,
                    end=end)
    assert f.calls == [(2, flags, 1234, 5678, 9)]


def test_last_piece_none(fake):
    ch, f = fake
    ch.chunk_device(np.array([16], dtype=np.uint64), [100], None, 1, 2)
    assert f.calls == [(1, 0, 1, 2, None)]
