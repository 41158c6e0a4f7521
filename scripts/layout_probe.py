"""Diagnostic: the tile kernel's read rate per stream layout over ONE allocation.  The same
64 GiB arena (config 2's bytes) is chunked as 1024 x 64 MiB streams (config 2), 64 x 1 GiB,
16 x 4 GiB and one 64 GiB stream (3 ii's shape); each layout's tile kernel time against the
bytes it must read (rc_keys_needed per stream).  Layouts alternate round after round.

    python scripts/layout_probe.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams, read_probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
MN, MX = 128_000, 5_120_000
TOTAL = 64 << 30
hs = torch.cuda.current_stream().cuda_stream
pool = torch.empty(TOTAL + 64, dtype=torch.uint8, device='cuda')
fill_splitmix_streams(pool.data_ptr(), 1024, 64 << 20, 64 << 20, synth.DEFAULT_SEED, 0, 1, hs)
ch = GpuChunker(MN, MX, b'\xff' * 16)
layouts = {'1024x64MiB': 1024, '64x1GiB': 64, '16x4GiB': 16, '1x64GiB': 1}
bufs = {}
for name, n in layouts.items():
    size = TOTAL // n
    total, caps = ch.capacity([size] * n)
    bufs[name] = (n, size, torch.zeros(total, dtype=torch.int64, device='cuda'),
                  torch.zeros(n, dtype=torch.int64, device='cuda'))
out = torch.zeros(4, dtype=torch.int32, device='cuda')


def needed(size):  # bytes up to the last key an argmax window reaches (L - max_length + 8)
    return min(size, size - MX + 8) if size > 2 * MX else size


res = {k: [] for k in layouts}
probe = []
for r in range(rounds):
    for name in (list(layouts) if r % 2 == 0 else list(layouts)[::-1]):
        n, size, cuts, counts = bufs[name]
        ptrs = [pool.data_ptr() + i * size for i in range(n)]
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(True)
        for _ in range(5):
            ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        res[name].append(t / k)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(3):
        read_probe(pool.data_ptr(), TOTAL, out.data_ptr(), hs)
    ev1.record()
    torch.cuda.synchronize()
    probe.append(3 * TOTAL / (ev0.elapsed_time(ev1) * 1e-3) / 1e9)
row = {'rounds': rounds, 'read_probe_gbs': round(float(np.median(probe)), 1)}
for name, v in res.items():
    n, size = layouts[name], TOTAL // layouts[name]
    ms = float(np.median(v))
    nb = n * needed(size)
    row[name] = {'tile_ms': round(ms, 4), 'bytes_needed': nb, 'read_gbs': round(nb / (ms * 1e-3) / 1e9, 1)}
print(json.dumps(row), flush=True)
