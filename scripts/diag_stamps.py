"""Diagnostic: per-step stamps of stream 0's chain walker (needs diag/lib_STAMPS.so)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['RC_LIB_PATH'] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'diag', 'lib_STAMPS.so')
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import _lib, synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

# usage: diag_stamps.py [n_streams] [stream_mib] [min] [max]   (default: config 2)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
size = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 20
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 128_000
mx = int(sys.argv[4]) if len(sys.argv) > 4 else 5_120_000
ch = GpuChunker(mn, mx, b'\xff' * 16)
pool = torch.empty(n * size, dtype=torch.uint8, device='cuda')
ptrs = [pool.data_ptr() + i * size for i in range(n)]
hs = torch.cuda.current_stream().cuda_stream
fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
total, caps = ch.capacity([size] * n)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
L = _lib.lib()
L.rc_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
for rep in range(3):
    ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    buf = np.zeros(4096, np.uint64)
    k = ctypes.c_uint32()
    L.rc_diag_read(buf.ctypes.data, 4096, ctypes.byref(k))
    v = buf[:k.value]
    tags = (v >> np.uint64(56)).astype(int)
    t = (v & np.uint64((1 << 56) - 1)).astype(np.int64)
    # per step: 1 start, 2 records done, 3 edges done, 4 step done
    d = {}
    for a, b in zip(range(len(t) - 1), range(1, len(t))):
        d.setdefault((tags[a], tags[b]), []).append((t[b] - t[a]) * 10)  # ns (100 MHz)
    print(f'rep {rep}: {k.value} stamps, span {(t[-1] - t[0]) * 10 / 1000:.1f} us')
    for key, vals in sorted(d.items()):
        print(f'  {key}: n={len(vals)} mean {np.mean(vals) / 1000:.2f} us  max {np.max(vals) / 1000:.2f}')
