"""Diagnostic: what config 3 (iii)'s tile kernel pays for, on ONE 64 GiB arena in one process:
the same bytes as 65,536 x 1 MiB streams (3 iii) or 1024 x 64 MiB, each with a small-window
chunker (min 2,000 / max 80,000) that writes group records (rc_tile_kernel<4>, the default for
such windows) and one built with RC_TILE_GROUPS=0 (rc_tile_kernel<1>); settings alternate
round after round, tile-kernel time by HIP events (sequential calls).

    python scripts/groups_ab.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
hs = torch.cuda.current_stream().cuda_stream
total = 64 << 30
pool = torch.empty(total + 64, dtype=torch.uint8, device='cuda')
fill_splitmix_streams(pool.data_ptr(), 65536, 1 << 20, 1 << 20, synth.DEFAULT_SEED, 0, 1, hs)
layouts = {'3iii_1MiB': (65536, 1 << 20), 'long_64MiB': (1024, 64 << 20)}
chs = {'groups': GpuChunker(2_000, 80_000, b'\xff' * 16)}
os.environ['RC_TILE_GROUPS'] = '0'
chs['nogroups'] = GpuChunker(2_000, 80_000, b'\xff' * 16)
os.environ.pop('RC_TILE_GROUPS')
res = {}
for r in range(rounds):
    for lay, (n, size) in layouts.items():
        ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
        lens = np.full(n, size, dtype=np.uint64)
        last = np.zeros(n, dtype=np.uint64)
        for name, ch in (chs.items() if r % 2 == 0 else list(chs.items())[::-1]):
            tot, caps = ch.capacity([size] * n)
            cuts = torch.zeros(tot, dtype=torch.int64, device='cuda')
            counts = torch.zeros(n, dtype=torch.int64, device='cuda')
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)
            torch.cuda.synchronize()
            ch.timing(True)
            for _ in range(5):
                ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)
            torch.cuda.synchronize()
            ch.timing(False)
            t, e, c, k = ch.read_kernel_timing()
            res.setdefault(f'{lay}/{name}', []).append((t / k, c / k, int(counts.sum().item())))
out = {}
for key, v in res.items():
    a = np.array([x[:2] for x in v])
    out[key] = {'tile_ms': round(float(np.median(a[:, 0])), 4), 'chain_ms': round(float(np.median(a[:, 1])), 4),
                'cuts': v[-1][2]}
print(json.dumps(out), flush=True)
