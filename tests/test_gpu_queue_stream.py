"""Own-queue streams (rc_stream_create, replicat_amd.chunker.QueueStream): the process-wide pool
hands a released stream out again, pools it once however often it is released, and close()
takes a pooled stream out of the pool before destroying it; torch work runs on it."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

from replicat_amd.chunker import QueueStream  # noqa: E402


def test_pool_reuse_and_close():
    dev = torch.cuda.current_device()
    a = QueueStream.acquire(dev)
    assert a.handle
    a.release()
    a.release()  # idempotent
    assert QueueStream._pool[dev].count(a) == 1
    assert QueueStream.acquire(dev) is a
    c = QueueStream.acquire(dev)
    assert c is not a and c.handle != a.handle
    c.release()
    c.close()  # never used by torch: destroyed now, and out of the pool
    assert c not in QueueStream._pool[dev] and c.handle is None
    c.release()  # a closed stream is not pooled again
    assert c not in QueueStream._pool[dev]
    with torch.cuda.stream(a.torch):
        x = torch.full((4096,), 2, dtype=torch.int64, device='cuda')
        y = x * 3
    a.torch.synchronize()
    assert int(y.sum().item()) == 6 * 4096
    a.release()
